"""LDS bank-conflict model of the register-resident FFT's transposes (reg_pass).

Bank rules (MI355X_MICROARCH.md, LDS table): ds_read_b64 is serviced in two 32-lane
groups with bank = (a/4) mod 64; ds_write_b64 in four 16-lane groups with bank = (a/4)
mod 32.  Each extra distinct 8-byte address on a busy bank within a group adds a cycle.

    python tools/lds_banks.py          # extra cycles per symbol for pad() vs the XOR swizzle
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


def main():
    lay = layouts()
    print("logn  " + "  ".join(f"{k:>6}" for k in lay))
    for logn in range(5, 13):
        print(f"{logn:4d}  " + "  ".join(f"{model(logn, f):6d}" for f in lay.values()))
    return 0


if __name__ == "__main__":
    sys.exit(main())
