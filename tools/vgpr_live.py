"""VGPR liveness of one kernel in a device assembly file: where the register pressure peaks and
which values are live there (with the source line that defined each), to find what keeps a
kernel above an occupancy step.

    hipcc --offload-arch=gfx950 -O3 ... -gline-tables-only --cuda-device-only -S k.hip -o k.s
    python tools/vgpr_live.py k.s [kernel-substring] [top]

Backward dataflow over the machine CFG of the final assembly (labels, s_cbranch_*, s_branch),
at 32-bit register granularity.  Stores (ds_write*, global_store*, buffer_store*, scratch_store*)
and v_cmp (SGPR / VCC destinations) only read VGPRs; v_writelane and the accumulating v_*fmac*
read their destination too.  Prints the peak, the instructions near it and the live set grouped by defining source
line.
"""

import re
import sys
from collections import Counter, defaultdict

REG = re.compile(r"\b([vs])(?:\[(\d+):(\d+)\]|(\d+)\b)")  # (no \b after "]": ranges were missed)
NODEF = re.compile(r"^(ds_write|ds_bpermute_b32_no|global_store|buffer_store|scratch_store|flat_store|"
                   r"v_cmp|v_cmpx|s_|exp|ds_gws|global_atomic(?!.*glc)|buffer_atomic(?!.*glc))")


def regs(text, kind="v"):
    out = []
    for m in REG.finditer(text):
        if m.group(1) != kind:
            continue
        if m.group(4) is not None:
            out.append(int(m.group(4)))
        else:
            out.extend(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def parse(path, filt):
    lines = open(path).read().split("\n")
    files, loc = {}, None
    body, on = [], False
    for ln in lines:
        m = re.match(r'\s+\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', ln)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
        if re.match(r"^_Z\S*:", ln):
            on = filt in ln
            continue
        if not on:
            continue
        m = re.match(r"\s+\.loc\s+(\d+)\s+(\d+)", ln)
        if m:
            loc = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
            continue
        if re.match(r"^\.LBB\d+_\d+:", ln):
            body.append(("label", ln.split(":")[0], loc))
            continue
        s = ln.split(";")[0].strip()
        if ln.startswith(".Lfunc_end"):
            on = False
            continue
        if not s or s.startswith("."):
            continue
        if re.match(r"^[a-z_0-9]+", s):
            body.append(("ins", s, loc))
    return body


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else "k_tx"
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    body = parse(path, filt)
    # basic blocks
    blocks, labels, cur = [], {}, None
    for kind, txt, loc in body:
        if kind == "label":
            cur = {"label": txt, "ins": [], "succ": []}
            labels[txt] = len(blocks)
            blocks.append(cur)
            continue
        if cur is None or (cur["ins"] and cur.get("term")):
            cur = {"label": None, "ins": [], "succ": []}
            blocks.append(cur)
        cur["ins"].append((txt, loc))
        op = txt.split()[0]
        if op.startswith("s_cbranch") or op == "s_branch" or op == "s_endpgm" or op.startswith("s_setpc"):
            cur["term"] = True
    for i, b in enumerate(blocks):
        if not b["ins"]:
            b["succ"] = [i + 1] if i + 1 < len(blocks) else []
            continue
        last = b["ins"][-1][0]
        op = last.split()[0]
        tgt = last.split()[1] if len(last.split()) > 1 else None
        if op == "s_branch":
            b["succ"] = [labels[tgt]]
        elif op.startswith("s_cbranch"):
            b["succ"] = [labels[tgt]] + ([i + 1] if i + 1 < len(blocks) else [])
        elif op == "s_endpgm" or op.startswith("s_setpc"):
            b["succ"] = []
        else:
            b["succ"] = [i + 1] if i + 1 < len(blocks) else []

    def du(txt):
        op = txt.split()[0]
        ops = txt[len(op):].strip()
        parts = [p.strip() for p in ops.split(",")]
        if NODEF.match(op) or not parts or not parts[0]:
            return set(), set(regs(ops))
        d = set(regs(parts[0]))
        u = set(regs(",".join(parts[1:])))
        if op.startswith("v_writelane") or "_dpp" in op or "fmac" in op or "_mac_" in op:
            u |= d  # partial write (other lanes keep their values) or an accumulating destination
        return d, u

    info = [[du(t) for t, _ in b["ins"]] for b in blocks]
    live_in = [set() for _ in blocks]
    changed = True
    while changed:
        changed = False
        for i in range(len(blocks) - 1, -1, -1):
            out = set()
            for s in blocks[i]["succ"]:
                out |= live_in[s]
            live = set(out)
            for d, u in reversed(info[i]):
                live -= d
                live |= u
            if live != live_in[i]:
                live_in[i] = live
                changed = True
    # per-instruction live-after sets; definitions' source lines
    defloc = defaultdict(Counter)
    for b in blocks:
        for (t, loc), (d, _) in zip(b["ins"], du_list(b, du)):
            for r in d:
                defloc[r][loc] += 1
    peak, where = -1, None
    profile = []
    for i, b in enumerate(blocks):
        out = set()
        for s in b["succ"]:
            out |= live_in[s]
        live = set(out)
        rows = []
        for k in range(len(b["ins"]) - 1, -1, -1):
            d, u = info[i][k]
            n = len(live | d)
            rows.append((k, n, set(live | d)))
            live -= d
            live |= u
        for k, n, ls in rows:
            profile.append(n)
            if n > peak:
                peak, where = n, (i, k, ls)
    i, k, ls = where
    print(f"peak live VGPRs {peak} at block {blocks[i]['label']} ins {k}: {blocks[i]['ins'][k][0]}  ({blocks[i]['ins'][k][1]})")
    for j in range(max(0, k - 4), min(len(blocks[i]["ins"]), k + 3)):
        print("   ", blocks[i]["ins"][j][0], " ", blocks[i]["ins"][j][1])
    # attribute each live register to its nearest preceding definition in program order (straight-
    # line code: the reaching definition; registers are reused, so "the line that most often
    # defines it" misleads)
    flat = [(bi, ki) for bi, b in enumerate(blocks) for ki in range(len(b["ins"]))]
    pos = flat.index((i, k))
    groups = Counter()
    for r in ls:
        src = "(entry / loop-carried)"
        for q in range(pos, -1, -1):
            bi, ki = flat[q]
            if r in info[bi][ki][0]:
                src = blocks[bi]["ins"][ki][1]
                break
        groups[src] += 1
    print("live set by reaching (nearest preceding) definition's source line:")
    for loc, n in groups.most_common(top):
        print(f"   {n:4d}  {loc}")


def du_list(b, du):
    return [du(t) for t, _ in b["ins"]]


if __name__ == "__main__":
    main()
