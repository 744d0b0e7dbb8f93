"""ctypes binding of ``libofdm_hip.so`` (C ABI: ``include/ofdm_hip.h``).

PyTorch-ROCm provides device memory and streams; every arithmetic step of the
modem path runs in the gfx950 kernels of the library.  There is no CPU fallback:
if the library or a GPU is missing, :func:`lib` / :func:`device` raise
:class:`BackendUnavailable`.

``import torch`` must happen before the library is loaded so that both share
torch's HIP runtime (``libamdhip64.so.7``) and therefore its streams.
"""

from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import numpy as np
import torch

# OFDM_LIB_VARIANT selects an alternative in-tree build (_lib/libofdm_hip_<variant>.so) for
# A/B timing studies; unset = the production library.
_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib",
                         "libofdm_hip%s.so" % ("_" + os.environ["OFDM_LIB_VARIANT"]
                                               if os.environ.get("OFDM_LIB_VARIANT") else ""))
# ABI 5: throughput-mode stream version 3 (the noise radius takes the whole lane word, the phase
# its own word per four samples; csrc/ofdm_device.hpp "throughput-mode streams")
ABI_VERSION = 5

OFDM_F32, OFDM_F64 = 0, 1
# ofdm_stats (include/ofdm_hip.h): power_sum, x_power_sum, x_peak (double), power_fx[2] (int64)
STATS_WORDS = 5
FX_HI, FX_LO = 2.0 ** -8, 2.0 ** -40
EQ_NONE, EQ_ZF, EQ_MMSE = 0, 1, 2
PREFIX_CYCLIC, PREFIX_ZERO = 0, 1
MOD_OFDM, MOD_SC = 0, 1

_c_i32p = ctypes.POINTER(ctypes.c_int32)
_c_f64p = ctypes.POINTER(ctypes.c_double)


class BackendUnavailable(RuntimeError):
    """The HIP library or a GPU is not available (the product has no CPU fallback)."""


class OfdmError(RuntimeError):
    """A libofdm_hip call returned an error code."""


class Desc(ctypes.Structure):
    _fields_ = [
        ("n_fft", ctypes.c_int32),
        ("cp", ctypes.c_int32),
        ("prefix", ctypes.c_int32),
        ("precision", ctypes.c_int32),
        ("equalizer", ctypes.c_int32),
        ("n_luts", ctypes.c_int32),
        ("lut_orders", _c_i32p),
        ("lut_pool", _c_f64p),
        ("sc_lut", _c_i32p),
        ("n_taps", ctypes.c_int32),
        ("h_raw", _c_f64p),
        ("H", _c_f64p),
        ("modulator", ctypes.c_int32),
    ]


class PlanInfo(ctypes.Structure):
    _fields_ = [
        ("n_fft", ctypes.c_int32),
        ("cp", ctypes.c_int32),
        ("precision", ctypes.c_int32),
        ("equalizer", ctypes.c_int32),
        ("n_taps", ctypes.c_int32),
        ("bits_per_ofdm_symbol", ctypes.c_int32),
        ("bits_per_subcarrier", ctypes.c_int32),
        ("adaptive", ctypes.c_int32),
        ("channel_gain_mean", ctypes.c_double),
    ]


# (name, restype, argtypes) -- mirrors include/ofdm_hip.h
_VP, _I32, _I64, _U64, _F64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
SIGNATURES = {
    "ofdm_abi_version": (ctypes.c_int, []),
    "ofdm_last_error": (ctypes.c_char_p, []),
    "ofdm_plan_create": (ctypes.c_int, [ctypes.POINTER(_VP), ctypes.POINTER(Desc), _VP]),
    "ofdm_plan_destroy": (ctypes.c_int, [_VP]),
    "ofdm_plan_get_info": (ctypes.c_int, [_VP, ctypes.POINTER(PlanInfo)]),
    "ofdm_plan_response": (ctypes.c_int, [_VP, _VP, _VP, _VP]),
    "ofdm_fft": (ctypes.c_int, [_VP, _VP, _VP, _I64, _I32]),
    "ofdm_map": (ctypes.c_int, [_VP, _VP, _VP, _I64, _I64, _VP]),
    "ofdm_demap": (ctypes.c_int, [_VP, _VP, _VP, _I64, _VP]),
    "ofdm_demap_count": (ctypes.c_int, [_VP, _VP, _VP, _VP, _I64, _VP]),
    "ofdm_nn_classify": (ctypes.c_int, [_VP, _VP, _I32, _VP, _I64, _VP]),
    "ofdm_noise_radius": (ctypes.c_int, [_VP, _VP, _I64, _VP]),
    "ofdm_modulate": (ctypes.c_int, [_VP, _VP, _VP, _I64, _VP]),
    "ofdm_demodulate": (ctypes.c_int, [_VP, _VP, _VP, _I64, _F64, _VP]),
    "ofdm_equalize": (ctypes.c_int, [_VP, _VP, _VP, _I64, _F64, _VP]),
    "ofdm_channel": (ctypes.c_int, [_VP, _VP, _VP, _I64, _VP, _VP]),
    "ofdm_awgn": (ctypes.c_int, [_VP, _VP, _VP, _I64, _VP, _VP, _VP, _F64]),
    "ofdm_power": (ctypes.c_int, [_VP, _VP, _VP, _I64, _VP]),
    "ofdm_tx": (ctypes.c_int, [_VP, _VP, _VP, _U64, _I64, _I64, _VP, _VP]),
    "ofdm_rx": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _U64, _VP, _I64, _F64, _I32, _VP, _I64, _I64,
                               _I64, _VP, _VP, _I64]),
}

_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()


def lib_path() -> str:
    return _LIB_PATH


def build_id() -> str:
    """Identity of the kernel sources the library is built from: sha256 (16 hex digits) over the
    HIP sources, the C-ABI header and the Makefile.  Profiles record it (profiles/pmc_summary.json)
    so that bench.py reports PMC traffic only for the build it was measured on."""
    import hashlib

    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # ofdm-based-systems_amd/
    root = os.path.dirname(pkg)
    files = sorted(os.path.join(pkg, "csrc", f) for f in os.listdir(os.path.join(pkg, "csrc")))
    files += [os.path.join(root, "include", "ofdm_hip.h"), os.path.join(pkg, "Makefile")]
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def load_library() -> ctypes.CDLL:
    """Load the library and bind every symbol of the header (no GPU needed)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(_LIB_PATH):
            raise BackendUnavailable(
                f"{_LIB_PATH} is missing: build it with `make -C ofdm-based-systems_amd` "
                "or __graft_entry__.build()")
        handle = ctypes.CDLL(_LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        # (a variant build of an earlier round -- same entry points, earlier stream version -- is
        # accepted for A/B studies when OFDM_LIB_VARIANT_ABI names its version)
        want = ABI_VERSION
        if os.environ.get("OFDM_LIB_VARIANT") and os.environ.get("OFDM_LIB_VARIANT_ABI"):
            want = int(os.environ["OFDM_LIB_VARIANT_ABI"])
        if handle.ofdm_abi_version() != want:
            raise BackendUnavailable("libofdm_hip ABI version mismatch")
        _lib = handle
        return handle


def device() -> torch.device:
    """The current HIP device; raises when no GPU is visible (no CPU fallback)."""
    if not torch.cuda.is_available():
        raise BackendUnavailable(
            "ofdm_based_systems runs its modem path on an AMD GPU (HIP); no GPU is visible")
    return torch.device("cuda", torch.cuda.current_device())


def lib() -> ctypes.CDLL:
    """Library handle for compute calls: requires both the .so and a GPU."""
    handle = load_library()
    device()
    return handle


def check(rc: int) -> None:
    """Raise on a non-zero return code: OFDM_E_INVALID -> ValueError (the reference's
    exception type for bad arguments), HIP / allocation failures -> OfdmError."""
    if rc != 0:
        msg = load_library().ofdm_last_error().decode(errors="replace")
        if rc == -1:
            raise ValueError(msg)
        raise OfdmError(f"libofdm_hip error {rc}: {msg}")


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def to_device(a: np.ndarray, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    a = np.ascontiguousarray(a)
    if not a.flags.writeable:  # e.g. np.frombuffer(bytes): torch wants a writable array
        a = a.copy()
    t = torch.from_numpy(a)
    if dtype is not None:
        t = t.to(dtype)
    return t.to(device(), non_blocking=False)


def _as_f64_ptr(a: Optional[np.ndarray]):
    if a is None:
        return None
    return a.ctypes.data_as(_c_f64p)


class Plan:
    """RAII wrapper of ``ofdm_plan_t`` (one modem configuration)."""

    def __init__(self, n_fft: int, cp: int = 0, precision: int = OFDM_F64, equalizer: int = EQ_NONE,
                 luts: Optional[list] = None, sc_lut: Optional[np.ndarray] = None,
                 h_raw: Optional[np.ndarray] = None, H: Optional[np.ndarray] = None,
                 prefix: int = PREFIX_CYCLIC, modulator: int = MOD_OFDM):
        self._lib = lib()
        self._handle = ctypes.c_void_p()
        luts = luts or []
        # keep every host array alive for the duration of the (synchronous) create call
        orders = np.array([len(l) for l in luts], dtype=np.int32)
        pool = (np.ascontiguousarray(np.concatenate([np.asarray(l, np.complex128) for l in luts]))
                .view(np.float64) if luts else None)
        sc = None if sc_lut is None else np.ascontiguousarray(sc_lut, dtype=np.int32)
        h = None if h_raw is None else np.ascontiguousarray(np.asarray(h_raw, np.complex128)).view(np.float64)
        Hh = None if H is None else np.ascontiguousarray(np.asarray(H, np.complex128)).view(np.float64)
        d = Desc()
        d.n_fft = int(n_fft)
        d.cp = int(cp)
        d.prefix = int(prefix)
        d.modulator = int(modulator)
        d.precision = int(precision)
        d.equalizer = int(equalizer)
        d.n_luts = len(luts)
        d.lut_orders = orders.ctypes.data_as(_c_i32p) if luts else None
        d.lut_pool = _as_f64_ptr(pool)
        d.sc_lut = sc.ctypes.data_as(_c_i32p) if sc is not None else None
        d.n_taps = 0 if h is None else len(h) // 2
        d.h_raw = _as_f64_ptr(h)
        d.H = _as_f64_ptr(Hh)
        check(self._lib.ofdm_plan_create(ctypes.byref(self._handle), ctypes.byref(d), stream_ptr()))
        info = PlanInfo()
        check(self._lib.ofdm_plan_get_info(self._handle, ctypes.byref(info)))
        self.n_fft = info.n_fft
        self.cp = info.cp
        self.precision = info.precision
        self.bits_per_ofdm_symbol = info.bits_per_ofdm_symbol
        self.bits_per_subcarrier = info.bits_per_subcarrier
        self.adaptive = bool(info.adaptive)
        self.channel_gain_mean = info.channel_gain_mean

    @property
    def handle(self):
        return self._handle

    @property
    def cdtype(self) -> torch.dtype:
        return torch.complex64 if self.precision == OFDM_F32 else torch.complex128

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            try:
                self._lib.ofdm_plan_destroy(h)
            except Exception:
                pass
            self._handle = ctypes.c_void_p()
