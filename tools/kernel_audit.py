"""Static audit of the fused kernels in a device assembly file: registers, spills and the memory
instructions that can stall the symbol loop (global loads other than the channel samples,
vmcnt waits, scratch traffic).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -fno-slp-vectorize [-DOFDM_AB_ONLY] \\
        --cuda-device-only -S ofdm-based-systems_amd/csrc/ofdm_kernels_f32.hip -o k.s
    python tools/kernel_audit.py k.s [name-substring]
"""

import re
import subprocess
import sys


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    txt = open(path).read().split("\n")
    meta, cur = {}, None
    for line in txt:
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            cur = m.group(1)
        m = re.match(r"\s+\.(vgpr_count|vgpr_spill_count|sgpr_spill_count|group_segment_fixed_size):\s+(\d+)", line)
        if m and cur:
            meta.setdefault(cur, {})[m.group(1)] = int(m.group(2))
    starts = [i for i, line in enumerate(txt) if re.match(r"^_ZN4ofdm4k_(tx|rx)\S*:", line)]
    for s in starts:
        name = txt[s].split(":")[0]
        if filt and filt not in name:
            continue
        e = next(i for i in range(s, len(txt)) if "s_endpgm" in txt[i])
        body = txt[s:e]
        gl = sum("global_load" in x for x in body)
        vm = sum("vmcnt" in x for x in body)
        sc = sum("scratch_" in x for x in body)
        fl = sum(re.search(r"\sflat_(load|store)", x) is not None for x in body)
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        md = meta.get(name, {})
        print(f"{dem.replace('ofdm::', '')[:44]:44s} vgpr {md.get('vgpr_count', '?'):>3} "
              f"spill {md.get('vgpr_spill_count', '?'):>3}/{md.get('sgpr_spill_count', '?'):<2} "
              f"global_load {gl:3d} vmcnt {vm:3d} scratch {sc:2d} flat {fl}")


if __name__ == "__main__":
    main()
