"""The C-ABI boundary (include/ofdm_hip.h) on CPU: the library loads, exports every
declared symbol, and rejects bad descriptors with the reference's messages before
touching the GPU."""

import ctypes
import os
import re

import numpy as np
import pytest
from conftest import ROOT

from ofdm_based_systems import _backend as B

HEADER = os.path.join(ROOT, "include", "ofdm_hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ofdm_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = B.load_library()
    names = declared_functions()
    assert len(names) >= 18
    for n in names:
        assert hasattr(lib, n), n
        assert n in B.SIGNATURES, f"{n} has no ctypes signature"
    assert set(B.SIGNATURES) == set(names)


def test_abi_version():
    assert B.load_library().ofdm_abi_version() == B.ABI_VERSION


def _create(**kw):
    lib = B.load_library()
    d = B.Desc()
    d.n_fft = kw.get("n_fft", 64)
    d.cp = kw.get("cp", 0)
    d.prefix = kw.get("prefix", 0)
    d.precision = kw.get("precision", 1)
    d.equalizer = kw.get("equalizer", 0)
    d.n_luts = kw.get("n_luts", 0)
    d.n_taps = kw.get("n_taps", 0)
    h = ctypes.c_void_p()
    rc = lib.ofdm_plan_create(ctypes.byref(h), ctypes.byref(d), None)
    return rc, lib.ofdm_last_error().decode()


@pytest.mark.parametrize("kw,msg", [
    ({"n_fft": 3}, "power of two"),
    ({"n_fft": 8192}, "power of two"),
    ({"n_fft": 0}, "power of two"),
    ({"cp": -1}, "Prefix length must be a non-negative integer."),
    ({"n_fft": 8, "cp": 9}, "Input symbols length must be greater than prefix length."),
    ({"precision": 7}, "precision"),
    ({"equalizer": 5}, "equalizer"),
    ({"n_taps": 40}, "n_taps"),
    ({"prefix": 3}, "prefix"),
])
def test_invalid_descriptors_fail_before_the_gpu(kw, msg):
    rc, err = _create(**kw)
    assert rc == -1
    assert msg in err


def test_check_maps_invalid_to_valueerror():
    _create(n_fft=3)
    with pytest.raises(ValueError, match="power of two"):
        B.check(-1)


def test_product_has_no_cpu_fallback():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ofdm_based_systems.constellation.models import QAMConstellationMapper

    with pytest.raises(B.BackendUnavailable):
        QAMConstellationMapper(16).decode(np.zeros(4, np.complex128))


def test_product_library_has_no_ablation_switches():
    """The timing tools' OFDM_ABLATE_TX / _RX switches (work skipping inside the kernels) are
    compiled only into -DOFDM_ABLATION=1 builds: the product library never reads them."""
    with open(B.lib_path(), "rb") as f:
        blob = f.read()
    assert b"OFDM_ABLATE" not in blob


def test_ab_only_variant_reports_kernels_it_lacks():
    """OFDM_AB_ONLY experiment builds (tools/ab.sh variants) instantiate N = 1024..4096 only.  Every
    log2 N dispatch switch falls through to kOutOfRange, which such a build defines as kNotInBuild,
    and the ABI turns that into OFDM_E_INVALID "kernel not in this build" (ValueError in Python)
    instead of a HIP "invalid argument"; a product build keeps hipErrorInvalidValue there (N is
    checked at plan creation, so it is never reached).  Checked on the sources, with the
    preprocessor branches evaluated both ways."""
    csrc = os.path.join(ROOT, "ofdm-based-systems_amd", "csrc")
    inst = open(os.path.join(csrc, "ofdm_kernels_inst.hpp")).read()
    launch = open(os.path.join(csrc, "ofdm_launch.hpp")).read()
    abi = open(os.path.join(csrc, "ofdm_abi.hip")).read()
    switches = re.findall(r"switch \(logn\) \{.*?default:\s*return (\w+);", inst, flags=re.S)
    assert len(switches) == 3 and set(switches) == {"kOutOfRange"}, switches

    def branch(text, name, ab_only):
        m = re.search(r"#ifdef OFDM_AB_ONLY\n(.*?)#else\n(.*?)#endif", text[text.index(name) - 200:], flags=re.S)
        return m.group(1 if ab_only else 2)

    assert "kOutOfRange = kNotInBuild" in branch(inst, "constexpr hipError_t kOutOfRange", True)
    assert "kOutOfRange = hipErrorInvalidValue" in branch(inst, "constexpr hipError_t kOutOfRange", False)
    assert "kAbOnly = true" in branch(launch, "constexpr bool kAbOnly", True)
    assert "kAbOnly = false" in branch(launch, "constexpr bool kAbOnly", False)
    hipchk = abi[abi.index("#define HIPCHK"):abi.index("} while (0)", abi.index("#define HIPCHK"))]
    assert "kAbOnly && _e == kNotInBuild" in hipchk and "OFDM_E_INVALID" in hipchk
    assert "kernel not in this build" in hipchk
