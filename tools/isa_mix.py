"""Static instruction mix of one kernel in a device assembly file, weighted by the measured
gfx950 issue costs (tools/isa_rates.hip).

    hipcc --offload-arch=gfx950 -O3 ... --cuda-device-only -S ofdm_kernels_f32.hip -o k.s
    python tools/isa_mix.py k.s '_ZN4ofdm4k_rxIfLi10ELin1ELi6EEEvNS_6RxArgsE'

Prints per-opcode counts and weighted issue cycles, for the whole kernel and for the
body of its innermost loops (blocks between a label and a backward branch to it).  With an
assembly built with -gline-tables-only, a third argument `lines` also attributes the
weighted cost to source lines (innermost inlined location of each instruction).
"""

import re
import sys
from collections import Counter

COST = [
    (r"^v_(log|exp|sqrt|rsq|rcp|sin|cos)_f32", 3.4),
    (r"^v_mad_u64_u32|^v_mad_i64_i32", 2.2),
    (r"^v_pk_(add|mul|fma)_f32", 1.9),
    (r"^v_fma_f32", 1.25),
    (r"^v_(cvt|bfe|perm|alignbit|alignbyte|med3|max_f32|min_f32|bcnt|add3|lshl_or|lshl_add|"
     r"add_lshl|mul_lo|mul_hi|mul_u32_u24|mad_u32_u24|and_or|or3|xad|ldexp|frexp|fract|cndmask|readlane|readfirstlane|writelane)", 1.7),
    (r"^v_", 1.0),
]


def cost(op):
    for pat, c in COST:
        if re.match(pat, op):
            return c
    return 0.0


def main():
    path, name = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end") or lines[i].strip() == "s_endpgm")
    body = lines[start:end + 1]
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', l)
        if m:
            files[int(m.group(1))] = m.group(2) + "/" + m.group(3)
    labels = {}
    ops = []  # (index, opcode)
    loc = None
    where = []
    for l in body:
        s = l.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            loc = (int(m.group(1)), int(m.group(2)))
            continue
        if not s or s.startswith(";") or s.startswith("."):
            m = re.match(r"^(\.LBB\w+):", s)
            if m:
                labels[m.group(1)] = len(ops)
            continue
        op = s.split()[0]
        ops.append((op, s))
        where.append(loc)
    loops = []
    for i, (op, s) in enumerate(ops):
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] <= i:
                loops.append((labels[tgt], i))
    def report(title, seq):
        c = Counter(op for op, _ in seq)
        tot = sum(cost(op) * n for op, n in c.items())
        nv = sum(n for op, n in c.items() if op.startswith("v_"))
        print(f"== {title}: {len(seq)} instr, {nv} VALU, weighted VALU issue {tot:.0f}")
        for op, n in sorted(c.items(), key=lambda x: -cost(x[0]) * x[1] - 1e-3 * x[1])[:40]:
            print(f"   {op:28s} {n:6d}  {cost(op) * n:8.1f}")
    report("kernel", ops)
    if len(sys.argv) > 3 and sys.argv[3] == "blocks":
        inv = sorted((v, k) for k, v in labels.items())
        bounds = [(0, "entry")] + inv + [(len(ops), "end")]
        print("== weighted VALU issue per basic block")
        for (a, na), (b, _) in zip(bounds[:-1], bounds[1:]):
            seq = ops[a:b]
            w = sum(cost(op) for op, _ in seq)
            tail = seq[-1][1] if seq else ""
            print(f"   {na:14s} [{a:5d},{b:5d})  {w:8.1f}   ends: {tail[:60]}")
    for a, b in loops:
        report(f"loop [{a}, {b}]", ops[a:b + 1])
    if len(sys.argv) > 3 and sys.argv[3] == "lines":
        per = Counter()
        for (op, _), w in zip(ops, where):
            per[w] += cost(op)
        src = {}
        print("== weighted VALU issue per source line")
        for w, c in per.most_common(45):
            if w is None or c == 0:
                continue
            f = files.get(w[0], "?")
            if f not in src:
                try:
                    src[f] = open(f).read().split("\n")
                except OSError:
                    src[f] = []
            text = src[f][w[1] - 1].strip() if 0 < w[1] <= len(src[f]) else ""
            print(f"   {c:7.1f}  {f.split('/')[-1]}:{w[1]:<5d} {text[:90]}")


if __name__ == "__main__":
    main()
