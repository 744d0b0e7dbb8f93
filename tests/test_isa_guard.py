"""Static guards on the built gfx950 code (CPU: disassembles libofdm_hip.so's device code objects
with the ROCm llvm-objdump; no GPU).

* No buffer stores anywhere in the device code.  A `buffer_store_dwordx4` with a register SGPR
  offset corrupted the low data dword of the window-FIR TX's last store on gfx950 (the compiler
  inserted no wait state between that store and the next VALU write of its data VGPRs; DESIGN.md
  section 4, profiles/r04g_diag_tx_determinism_e.txt); every store of the product kernels is a
  global_store, and this keeps it that way.
* The split FFT exchange's inline-assembly reads (ds_read16_b64: 16 `ds_read_b64` and their
  `s_waitcnt lgkmcnt(0)` in one statement) reach the ISA as an uninterrupted run of 16 reads
  followed directly by the wait: the compiler does not track inline-assembly LDS loads, so any
  instruction between a read and the wait could see a stale destination.
"""

import os
import re
import struct
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

from ofdm_based_systems import _backend as B

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
OBJCOPY = "/opt/rocm/lib/llvm/bin/llvm-objcopy"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _code_objects(lib_path, tmp):
    """The gfx950 code objects of the library's .hip_fatbin section (clang offload bundles:
    magic, u64 entry count, then per entry u64 offset, u64 size, u64 triple length, triple)."""
    fat = os.path.join(tmp, "fatbin.bin")
    subprocess.run([OBJCOPY, f"--dump-section=.hip_fatbin={fat}", lib_path, os.path.join(tmp, "stripped.so")],
                   check=True, capture_output=True)
    blob = open(fat, "rb").read()
    out = []
    i = blob.find(MAGIC)
    while i >= 0:
        (n,) = struct.unpack_from("<Q", blob, i + len(MAGIC))
        p = i + len(MAGIC) + 8
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "gfx950" in triple and size > 0:
                out.append(blob[i + off:i + off + size])
        i = blob.find(MAGIC, i + len(MAGIC))
    return out


@pytest.fixture(scope="module")
def disassembly(tmp_path_factory):
    if not (os.path.exists(OBJDUMP) and os.path.exists(OBJCOPY)):
        pytest.skip("ROCm llvm tools not present")
    tmp = str(tmp_path_factory.mktemp("isa"))
    objs = _code_objects(B.lib_path(), tmp)
    assert objs, "no gfx950 code object in the library"
    paths = []
    for k, o in enumerate(objs):
        p = os.path.join(tmp, f"co{k}.elf")
        with open(p, "wb") as f:
            f.write(o)
        paths.append(p)

    def dis(p):
        return subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", p], check=True, capture_output=True,
                              text=True).stdout

    with ThreadPoolExecutor(max_workers=min(8, len(paths))) as ex:
        return list(ex.map(dis, paths))


def _functions(text):
    """{symbol: [instruction lines]} of one objdump listing."""
    funcs, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        s = line.strip()
        if cur is not None and s and not s.startswith(";"):
            cur.append(s.split("//")[0].strip())
    return funcs


def test_fused_kernels_are_present(disassembly):
    names = [n for t in disassembly for n in _functions(t)]
    assert any(n.startswith("_ZN4ofdm4k_txI") for n in names)
    assert any(n.startswith("_ZN4ofdm4k_rxI") for n in names)


def test_no_buffer_stores_in_device_code(disassembly):
    bad = []
    for t in disassembly:
        for name, ins in _functions(t).items():
            bad += [(name, x) for x in ins if x.startswith("buffer_store")]
    assert not bad, bad[:5]


def test_inline_lds_reads_wait_in_one_block(disassembly):
    """A ds_read16_b64 block: 16 consecutive ds_read_b64 off one address register (the compiler pairs
    its own reads into ds_read2_b64), then s_waitcnt lgkmcnt(0) at once."""
    rd = re.compile(r"^ds_read_b64 v\[\d+:\d+\], (v\d+)(?: offset:\S+)?$")
    blocks = 0
    for t in disassembly:
        for name, ins in _functions(t).items():
            if not name.startswith(("_ZN4ofdm4k_txI", "_ZN4ofdm4k_rxI")):
                continue  # the fused kernels hold the split exchange
            addr = [(m.group(1) if m else None) for m in (rd.match(x) for x in ins)]
            k = 0
            while k + 16 <= len(ins):
                a = addr[k]
                if a is not None and all(addr[k + i] == a for i in range(16)):
                    blocks += 1
                    nxt = ins[k + 16] if k + 16 < len(ins) else ""
                    assert nxt.startswith("s_waitcnt") and "lgkmcnt(0)" in nxt, (name, ins[k + 14:k + 18])
                    k += 16
                else:
                    k += 1
    assert blocks > 0, "no inline 16-read exchange block found"
