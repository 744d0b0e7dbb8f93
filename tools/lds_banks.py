"""LDS bank-conflict model of the register-resident FFT's transposes (reg_pass).

Bank rules (MI355X_MICROARCH.md, LDS table): ds_read_b64 is serviced in two 32-lane
groups with bank = (a/4) mod 64; ds_write_b64 in four 16-lane groups with bank = (a/4)
mod 32.  Each extra distinct 8-byte address on a busy bank within a group adds a cycle.

    python tools/lds_banks.py          # extra cycles per symbol for pad() vs the XOR swizzle
    python tools/lds_banks.py --fir    # complex128 window-FIR TX rows: wfir_slot vs wfir_in / wfir_out

The --fir model covers the 16-byte accesses of the complex128 window FIR (ofdm_fused.hpp): the FFT
elements written into the half-symbol row (ds_write_b128: eight 8-lane groups, bank mod 32), the
lanes' windows read at lane stride 8 stream samples and the stores' read-back of the outputs
(ds_read_b128: four 16-lane groups {0-3,12-15,20-27}, ..., bank mod 64), and the outputs'
transpose writes.  It predicts 192 extra cycles per config-(c) symbol for the round-3/4 layout
(measured SQ_LDS_BANK_CONFLICT: 197, profiles/r04c_counters_c_f64.txt) and 0 for the current one.
"""

import sys


def geo(logn):
    E = 1 << min(4, logn)
    N = 1 << logn
    tps = N // E
    return N, E, tps, 256 // tps, N + N // 16 + 1


def passes(logn):
    out, logns = [], 0
    while logns < logn:
        logr = min(4, logn - logns)
        out.append((logr, logns))
        logns += logr
    return out


def layouts():
    return {
        "pad": lambda i: i + (i >> 4),
        "xor": lambda i: (i & ~15) | ((i & 15) ^ ((i >> 4) & 15)),
    }


def conflicts(addrs, group, modulus):
    """addrs: per lane element slot (8-byte units) -> extra cycles of one wave instruction."""
    extra = 0
    for g0 in range(0, 64, group):
        banks = {}
        for a in addrs[g0:g0 + group]:
            if a is None:
                continue
            b = (2 * a) % modulus  # first dword bank; an 8-byte element spans banks b, b+1
            banks.setdefault(b, set()).add(a)
        extra += max((len(v) for v in banks.values()), default=1) - 1
    return extra


def model(logn, slot):
    N, E, tps, spb, padn = geo(logn)
    rows = lambda lane: ((lane // tps) % spb) * padn  # symbol row base of a lane in wave 0
    total = 0
    for logr, logns in passes(logn):
        rad, ns = 1 << logr, 1 << logns
        nb, stride = E // rad, N // rad
        first, last = logns == 0, logns + logr == logn
        if not first:  # reads v[q][r] = buf[t + q*TPS + r*STRIDE]
            for q in range(nb):
                for r in range(rad):
                    addrs = [rows(l) + slot(l % tps + q * tps + r * stride) for l in range(64)]
                    total += conflicts(addrs, 32, 64)
        if not last:  # writes buf[idx + r*NS], idx = ((j >> LOGNS) << (LOGNS+LOGR)) + (j & (NS-1))
            for q in range(nb):
                for r in range(rad):
                    addrs = []
                    for l in range(64):
                        j = l % tps + q * tps
                        idx = ((j >> logns) << (logns + logr)) + (j & (ns - 1))
                        addrs.append(rows(l) + slot(idx + r * ns))
                    total += conflicts(addrs, 16, 32)
    return total


RG128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
         list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
RG128 += [[x + 32 for x in g] for g in RG128]
WG128 = [list(range(8 * k, 8 * k + 8)) for k in range(8)]


def conflicts16(slots, groups, mod):
    """16-byte accesses: slot s occupies the 4 banks of (s mod `mod`) (mod 8: writes, 16: reads)."""
    extra = 0
    for g in groups:
        seen, cnt = set(), {}
        for lane in g:
            s = slots[lane]
            if s in seen:
                continue  # same address: broadcast
            seen.add(s)
            cnt[s % mod] = cnt.get(s % mod, 0) + 1
        extra += max(cnt.values(), default=1) - 1
    return extra


def fir_model(slot_in, slot_out, lt=8, cp=7, logn=10):
    n = 1 << logn
    nh, so = n // 2, cp
    a8 = (so + 7) & ~7
    tot = {}
    for h in (0, 1):
        ah = a8 if h == 0 else 0
        b = ah - so - h * nh + (lt - 1)
        tot[f"x write h{h}"] = sum(conflicts16([slot_in(b + so + t + 64 * i) for t in range(64)], WG128, 8)
                                   for i in range(8 * h, 8 * h + 8))
        tot[f"window read h{h}"] = sum(conflicts16([slot_in(ah + 8 * t + w) for t in range(64)], RG128, 16)
                                       for w in range(8 + lt - 1))
        tot[f"y write h{h}"] = sum(conflicts16([slot_out(8 * t + j) for t in range(64)], WG128, 8) for j in range(8))
        tot[f"y read h{h}"] = sum(conflicts16([slot_out(t + 64 * i) for t in range(64)], RG128, 16) for i in range(8))
    return tot


def fir_main():
    old = lambda k: k + (k >> 3)
    for lt, cp in ((8, 7), (4, 3)):
        ioff = (9 - lt) & 7
        new_in = lambda k: k + ((k + ioff) >> 3)
        new_out = lambda k: (k & ~7) | ((k ^ (k >> 3)) & 7)
        for name, si, sout in (("wfir_slot", old, old), ("wfir_in/out", new_in, new_out)):
            t = fir_model(si, sout, lt, cp)
            print(f"LT={lt} cp={cp} {name:12s} extra cycles per symbol {sum(t.values()):4d}  {t}")
    return 0


def main():
    if "--fir" in sys.argv:
        return fir_main()
    lay = layouts()
    print("logn  " + "  ".join(f"{k:>6}" for k in lay))
    for logn in range(5, 13):
        print(f"{logn:4d}  " + "  ".join(f"{model(logn, f):6d}" for f in lay.values()))
    return 0


if __name__ == "__main__":
    sys.exit(main())
