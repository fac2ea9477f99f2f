#!/usr/bin/env python3
"""LDS bank-conflict model of the Stockham exchanges (kernels.hpp / fft_core.hpp)
for one plan and kernel geometry, to pick an exchange layout before building.

Per wave instruction (MI355X_MICROARCH.md, LDS table): ds_write_b64 is
serviced in 4 groups of 16 lanes on 32 banks ((dword) mod 32), ds_read_b64 in
2 groups of 32 lanes on 64 banks; a group costs max over banks of the distinct
dwords on that bank (identical addresses broadcast). Reported: extra cycles
per instruction over the conflict-free count (SQ_LDS_BANK_CONFLICT analogue).

    python tools/lds_banks.py            # every kernel geometry the bench runs
"""
import sys

PLANS = {  # plans.hpp kPlans: key -> (n, e, radices)
    5: (1024, 16, (16, 4, 16)), 11: (1024, 8, (8, 4, 4, 8)), 13: (4096, 16, (16, 16, 16)),
    8: (256, 8, (8, 4, 8)), 12: (2048, 8, (8, 4, 8, 8)), 10: (768, 12, (4, 12, 4, 4)),
}


def pad16(o):
    return o + (o >> 4)


def swz(o):
    """XOR swizzle: low 4 bits of the element index ^= bits 4..7 (no padding)."""
    return o ^ ((o >> 4) & 15)


def group_cost(dwords, banks):
    per = {}
    for d in set(dwords):
        per.setdefault(d % banks, set()).add(d)
    return max(len(v) for v in per.values()) if per else 0


def instr_cost(addrs, write):
    """addrs: 64 element (float2) addresses of one wave instruction (None = inactive)."""
    if write:
        extra = 0
        for g in range(4):
            dw = []
            for a in addrs[16 * g:16 * g + 16]:
                if a is not None:
                    dw += [2 * a, 2 * a + 1]
            extra += max(0, group_cost(dw, 32) - 1)
        return extra
    extra = 0
    for g in range(2):
        dw = []
        for a in addrs[32 * g:32 * g + 32]:
            if a is not None:
                dw += [2 * a, 2 * a + 1]
        extra += max(0, group_cost(dw, 64) - 1)
    return extra


def lane_map(kind, key, cw=2, rpw=2, L=1):
    """tid -> (t, line id) for the row / column kernels' lane mappings."""
    n, e, _ = PLANS[key]
    T = n // e
    out = []
    if kind == "row":
        rl = rpw // L
        tl = min(T, 16)
        qr = min(rl, 4)
        for tid in range(rl * T):
            tlo = tid % tl
            q4 = (tid // tl) % qr
            rest = tid // (qr * tl)
            qq = rest // (T // tl)
            t = tlo + tl * (rest - qq * (T // tl))
            out.append((t, (qq * qr + q4) * L))
    elif kind == "wave":  # one line per wave (T == 64 or T % 64 == 0: lines of T threads, contiguous lanes)
        for tid in range(rpw * T):
            out.append((tid % T, (tid // T) * L))
    else:
        for tid in range(cw // L * T):
            out.append((tid // (cw // L), (tid % (cw // L)) * L))
    return out


def simulate(kind, key, layout, cw=2, rpw=2, L=1):
    n, e, radices = PLANS[key]
    T = n // e
    lanes = lane_map(kind, key, cw, rpw, L)
    line = n + n // 16 if layout == "pad16" else n
    rowstride = line + ((16 - line % 32) + 32) % 32
    f = pad16 if layout in ("pad16", "pad16tile") else swz

    def addr(line_id, l, o):
        if kind in ("row", "wave"):
            return (line_id + l) * rowstride + f(o)
        if layout.endswith("tile") or layout == "pad16":
            return f(o) * cw + line_id + l
        return (line_id + l) * (n + 32) + f(o)  # line-major columns

    wr = rd = nw = nr = 0
    ns = 1
    for pi, R in enumerate(radices):
        nb = e // R
        last = pi == len(radices) - 1
        if not last:
            for k in range(nb):
                for l in range(L):
                    for r in range(R):
                        for w0 in range(0, len(lanes), 64):
                            a = []
                            for t, lid in lanes[w0:w0 + 64]:
                                b = t + k * T
                                j = b % ns
                                o = (b // ns) * ns * R + j + r * ns
                                a.append(addr(lid, l, o))
                            wr += instr_cost(a, True)
                            nw += 1
            for l in range(L):
                for m in range(e):
                    for w0 in range(0, len(lanes), 64):
                        a = [addr(lid, l, t + m * T) for t, lid in lanes[w0:w0 + 64]]
                        rd += instr_cost(a, False)
                        nr += 1
        ns *= R
    return wr / max(nw, 1), rd / max(nr, 1)


def main():
    cases = [("col 1024 narrow cw2", "col", 11, dict(cw=2)), ("row 1024 narrow pairs", "row", 11, dict(rpw=2)),
             ("col 4096 narrow cw2 L2", "col", 13, dict(cw=2, L=2)), ("row 4096 narrow single", "row", 13,
                                                                           dict(rpw=1)),
             ("col 1024 wide cw4", "col", 5, dict(cw=4)), ("row 1024 wide quads", "row", 5, dict(rpw=4)),
             ("row 1024 wide wave-line", "wave", 5, dict(rpw=4))]
    layouts = sys.argv[1:] or ["pad16", "swz", "swztile"]
    for name, kind, key, kw in cases:
        res = []
        for lay in layouts:
            try:
                w, r = simulate(kind, key, lay, **kw)
                res.append(f"{lay}: write {w:.2f} read {r:.2f}")
            except Exception as ex:  # noqa: BLE001
                res.append(f"{lay}: {ex}")
        print(f"{name:28s} " + " | ".join(res))


if __name__ == "__main__":
    main()


ALL = {0: (64, 8, (8, 8), 0), 1: (128, 16, (4, 8, 4), 0), 2: (256, 16, (16, 16), 0), 3: (512, 16, (16, 2, 16), 0),
       4: (768, 24, (8, 12, 8), 0), 5: (1024, 16, (16, 4, 16), 0), 6: (2048, 16, (16, 8, 16), 0),
       7: (4096, 32, (8, 8, 8, 8), 0), 8: (256, 8, (8, 4, 8), 1), 9: (512, 8, (8, 8, 8), 1),
       10: (768, 12, (4, 12, 4, 4), 1), 11: (1024, 8, (8, 4, 4, 8), 1), 12: (2048, 8, (8, 4, 8, 8), 1),
       13: (4096, 16, (16, 16, 16), 1)}


def row_rpw(key):
    n, e, _, var = ALL[key]
    T = n // e
    line = n + n // 16
    rs = line + ((16 - line % 32) + 32) % 32
    if T < 64:
        return 256 // T
    single = var == 1 and n >= 4096
    pairs = (4 * rs * 8 > 80 * 1024 and T >= 256) or var == 1
    return 1 if single else 2 if pairs else 4


def sweep():
    PLANS.update({k: v[:3] for k, v in ALL.items()})
    for key in ALL:
        n, e, rad, var = ALL[key]
        rr = [f"{lay}: " + "w %.2f r %.2f" % simulate("row", key, lay, rpw=row_rpw(key)) for lay in ("pad16", "swz")]
        print(f"row key {key:2d} n {n:4d} e {e:2d} {rad}: " + " | ".join(rr))
        for cw in (2, 4):
            L = 2 if (var == 1 and n >= 4096 and cw % 2 == 0) else 1
            if (cw // L) * (n // e) > 1024:
                continue
            cc = [f"{lay}: " + "w %.2f r %.2f" % simulate("col", key, lay, cw=cw, L=L) for lay in ("pad16", "swz")]
            print(f"   col cw {cw} L {L}: " + " | ".join(cc))
