"""LDS bank-conflict model of the mixed-radix passes (mixed_radix.hpp, `pass`).

Replays the complex128 LDS reads (ds_read_b128) and writes (ds_write_b128) of
every radix pass of one tile, lane by lane, with the lane groups and bank
functions of MI355X_MICROARCH.md (LDS table; the same model as
tools/lds_bank_sim.py, which matches the measured SQ_LDS_BANK_CONFLICT of the
relayout kernels), and prints the extra cycles per LDS instruction for a
layout function of the element index (plain, or padded by one slot per 16).
usage: python tools/mr_lds_sim.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lds_bank_sim import extra_cycles  # noqa: E402

THREADS = 256


def radices(n):
    out = []
    while n % 8 == 0:
        out.append(8)
        n //= 8
    for r in (4, 2, 3, 5, 7, 11, 13):
        while n % r == 0:
            out.append(r)
            n //= r
    assert n == 1
    return out


def passes(n, count, ls, es, linefast, lay):
    """(kind, words, 64 addresses) per wave-instruction of a DIF over the tile"""
    out = []
    L = n
    for R in radices(n):
        m = L // R
        per_line = n // R
        nb = count * per_line
        step = m * es
        for g0 in range(0, nb, THREADS):
            for w in range(THREADS // 64):
                bases = []
                for lane in range(64):
                    gi = g0 + w * 64 + lane
                    if gi >= nb:
                        bases.append(None)
                        continue
                    if linefast:
                        line, bf = gi % count, gi // count
                    else:
                        line, bf = gi // per_line, gi % per_line
                    blk, j = bf // m, bf % m
                    bases.append(line * ls + (blk * L + j) * es)
                for r in range(R):
                    addrs = [None if b is None else 4 * lay(b + r * step) for b in bases]  # 16 B = 4 words
                    out.append(("r", 4, addrs))
                    out.append(("w", 4, addrs))
        L = m
    return out


def main():
    plain = lambda e: e  # noqa: E731
    pad16 = lambda e: e + (e >> 4)  # noqa: E731
    pad8 = lambda e: e + (e >> 3)  # noqa: E731
    for n, count, what in ((1920, 1, "rows of 1920 (tile of 1 row)"), (1080, 2, "columns of 1080, tile of 2"),
                           (1080, 4, "columns of 1080, tile of 4"), (1024, 2, "columns of 1024, tile of 2"),
                           (1280, 1, "rows of 1280")):
        col = what.startswith("columns")
        geo = (count, 1, count, True) if col else (count, n, 1, False)
        res = []
        for name, lay in (("plain", plain), ("pad 1/16", pad16), ("pad 1/8", pad8)):
            acc = passes(n, *geo, lay)
            rd = [a for a in acc if a[0] == "r"]
            wr = [a for a in acc if a[0] == "w"]
            res.append(f"{name}: read {sum(extra_cycles(*a) for a in rd) / len(rd):.2f} "
                       f"write {sum(extra_cycles(*a) for a in wr) / len(wr):.2f}")
        print(f"{what:32s} " + " | ".join(res))


if __name__ == "__main__":
    main()
