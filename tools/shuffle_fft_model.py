#!/usr/bin/env python3
"""NumPy model of the wave-shuffle 1024-point transform pair (fft_shuffle.hpp).

Simulates one 256-thread workgroup (4 waves of 64 lanes, lane bit 0 selects
one of the two lines) holding 8 complex values per thread, and runs exactly
the passes, twiddles and exchanges the HIP engine runs:

  forward DIF  P1 (radix 8) - X1 permlane - P2 (4) - X2 LDS - P3 (4) - X3 permlane - P4 (8)
  middle       element-wise epilogue; slot m of thread tau holds frequency
               k = pos_load(tau, m), the same index the thread loaded
  inverse DIT  P4^H - X3 - P3^H - X2^H LDS - P2^H - X1 - P1^H

v_permlane16_swap / v_permlane32_swap are modelled by their ISA semantics
(swap odd 16-lane rows of vdst with even rows of src / upper half of vdst with
lower half of src). Checks the pair against numpy.fft and prints the LDS bank
conflicts of the X2 exchange under the slot swizzle.

    python tools/shuffle_fft_model.py
"""
import numpy as np

N, E, THREADS = 1024, 8, 256


def bit(x, i):
    return (x >> i) & 1


def pos_load(tid, m):
    lam, om = tid & 63, tid >> 6
    return ((lam >> 1) & 7) | (om << 3) | (((lam >> 4) & 3) << 5) | (m << 7)


def line_of(tid):
    return tid & 1


def pos_b(tid, m):
    """state after X1: slot bits (pos7, pos5, pos6), l1..l3 pos0-2, l4 pos8, l5 pos9, w pos3,4"""
    lam, om = tid & 63, tid >> 6
    p = ((lam >> 1) & 7) | (om << 3)
    p |= bit(m, 0) << 7 | bit(m, 1) << 5 | bit(m, 2) << 6
    p |= bit(lam, 4) << 8 | bit(lam, 5) << 9
    return p


def pos_c(tid, m):
    """state after X2: slot bits (pos3, pos4, pos2), l1..l3 pos7-9, l4 pos0, l5 pos1, w pos5,6"""
    lam, om = tid & 63, tid >> 6
    p = ((lam >> 1) & 7) << 7 | (om << 5)
    p |= bit(lam, 4) << 0 | bit(lam, 5) << 1
    p |= bit(m, 0) << 3 | bit(m, 1) << 4 | bit(m, 2) << 2
    return p


def pos_d(tid, m):
    """state after X3: slot bits (pos0, pos1, pos2), l4 pos3, l5 pos4"""
    lam, om = tid & 63, tid >> 6
    p = ((lam >> 1) & 7) << 7 | (om << 5)
    p |= bit(lam, 4) << 3 | bit(lam, 5) << 4
    p |= m
    return p


def permlane16_swap(a, b):
    """a, b: [THREADS] arrays (one VGPR); rows of 16 lanes per wave"""
    a, b = a.copy(), b.copy()
    for w in range(THREADS // 64):
        for r in (0, 2):
            lo = slice(w * 64 + r * 16, w * 64 + r * 16 + 16)
            hi = slice(w * 64 + (r + 1) * 16, w * 64 + (r + 1) * 16 + 16)
            a[hi], b[lo] = b[lo].copy(), a[hi].copy()
    return a, b


def permlane32_swap(a, b):
    a, b = a.copy(), b.copy()
    for w in range(THREADS // 64):
        lo = slice(w * 64, w * 64 + 32)
        hi = slice(w * 64 + 32, w * 64 + 64)
        a[hi], b[lo] = b[lo].copy(), a[hi].copy()
    return a, b


def swap_slots(v, sbit, which):
    """swap slot bit `sbit` with lane bit 4 (which=16) or 5 (which=32)"""
    f = permlane16_swap if which == 16 else permlane32_swap
    for m in range(E):
        if bit(m, sbit) == 0:
            v[:, m], v[:, m | (1 << sbit)] = f(v[:, m], v[:, m | (1 << sbit)])


def dft(u, inv):
    R = len(u)
    k = np.arange(R)
    w = np.exp((2j if inv else -2j) * np.pi * np.outer(k, k) / R)
    return w @ u


def root(e, inv):
    z = np.exp(-2j * np.pi * (e % N) / N).astype(np.complex64)
    return np.conj(z) if inv else z


# per-thread twiddle exponents of the three twiddled passes
def tw_p1(tid):  # w_1024^(n k1), n = pos & 127
    n = pos_load(tid, 0) & 127
    return [n * k for k in range(1, 8)]


def tw_p2(tid):  # w_128^(n k2) = w_1024^(8 n k2), n = pos & 31
    n = pos_load(tid, 0) & 31
    return [8 * n * k for k in range(1, 4)]


def tw_p3(tid, hi):  # w_32^(n k3) = w_1024^(32 n k3), n = pos0 + 2 pos1 + 4 pos2; pos2 = slot bit 2
    lam = tid & 63
    n = bit(lam, 4) | bit(lam, 5) << 1 | hi << 2
    return [32 * n * k for k in range(1, 4)]


def groups(kind):
    if kind == 1:
        return [[0, 1, 2, 3, 4, 5, 6, 7]]
    if kind == 2:  # digit over slot bits 1,2; butterflies by slot bit 0
        return [[b0 + 2 * d for d in range(4)] for b0 in range(2)]
    if kind == 3:  # digit over slot bits 0,1; butterflies by slot bit 2
        return [[4 * hi + d for d in range(4)] for hi in range(2)]
    return [[0, 1, 2, 3, 4, 5, 6, 7]]


def tw_of(tid, kind, g):
    if kind == 1:
        return tw_p1(tid)
    if kind == 2:
        return tw_p2(tid)
    if kind == 3:
        return tw_p3(tid, g)
    return None


def pass_dif(v, kind, inv):
    for tid in range(THREADS):
        for g, slots in enumerate(groups(kind)):
            u = dft(v[tid, slots].astype(np.complex128), inv)
            tw = tw_of(tid, kind, g)
            if tw is not None:
                for r in range(1, len(slots)):
                    u[r] *= root(tw[r - 1], inv)
            v[tid, slots] = u.astype(np.complex64)


def pass_dit(v, kind, inv):
    for tid in range(THREADS):
        for g, slots in enumerate(groups(kind)):
            u = v[tid, slots].astype(np.complex128)
            tw = tw_of(tid, kind, g)
            if tw is not None:
                for r in range(1, len(slots)):
                    u[r] *= root(tw[r - 1], inv)
            v[tid, slots] = dft(u, inv).astype(np.complex64)


def lds_exchange(v, src_pos, dst_pos):
    lds = {}
    for tid in range(THREADS):
        for m in range(E):
            lds[lds_slot(src_pos(tid, m), line_of(tid))] = v[tid, m]
    out = np.empty_like(v)
    for tid in range(THREADS):
        for m in range(E):
            out[tid, m] = lds[lds_slot(dst_pos(tid, m), line_of(tid))]
    return out


def lds_slot(p, line):
    """element slot of position p of a line (fft_shuffle.hpp, shuffle_slot): the
    low 5 bits are XORed with H(j = p >> 7, line), a bijection chosen so that
    both halves of both X2 directions are conflict-free"""
    j0, j1, j2 = bit(p, 7), bit(p, 8), bit(p, 9)
    h = j2 | j0 << 1 | j1 << 2 | (line ^ j2) << 3 | (j2 ^ j1) << 4
    return line * N + (p ^ h)


def bank_conflicts(pos_fn, kind):
    """extra LDS cycles of one exchange half under the tools/lds_banks.py model:
    8-B accesses, 64 banks of 4 B for ds_read_b64 (two 32-lane halves), 32 banks
    for ds_write_b64 (four 16-lane groups); address = line * 1024 + slot"""
    total = 0
    for w in range(THREADS // 64):
        for m in range(E):
            lanes = range(w * 64, w * 64 + 64)
            addr = [2 * lds_slot(pos_fn(t, m), line_of(t)) for t in lanes]  # dword address
            grp, nb = (32, 64) if kind == "read" else (16, 32)
            for g0 in range(0, 64, grp):
                banks = {}
                for a in addr[g0:g0 + grp]:
                    for d in (a, a + 1):
                        banks.setdefault(d % nb, set()).add(d)
                total += max(len(s) for s in banks.values()) - 1
    return total


def run_pair(x, col_like=True):
    """x: [2 lines][N]; col_like: forward then inverse (column pass) else inverse then forward"""
    v = np.empty((THREADS, E), np.complex64)
    for tid in range(THREADS):
        for m in range(E):
            v[tid, m] = x[line_of(tid), pos_load(tid, m)]
    inv1 = not col_like
    pass_dif(v, 1, inv1)
    swap_slots(v, 1, 16)
    swap_slots(v, 2, 32)
    pass_dif(v, 2, inv1)
    v = lds_exchange(v, pos_b, pos_c)
    pass_dif(v, 3, inv1)
    swap_slots(v, 0, 16)
    swap_slots(v, 1, 32)
    pass_dif(v, 4, inv1)
    mid = np.empty_like(x)
    for tid in range(THREADS):
        for m in range(E):
            mid[line_of(tid), pos_load(tid, m)] = v[tid, m]
    inv2 = col_like
    pass_dit(v, 4, inv2)
    swap_slots(v, 0, 16)
    swap_slots(v, 1, 32)
    pass_dit(v, 3, inv2)
    v = lds_exchange(v, pos_c, pos_b)
    pass_dit(v, 2, inv2)
    swap_slots(v, 1, 16)
    swap_slots(v, 2, 32)
    pass_dit(v, 1, inv2)
    out = np.empty_like(x)
    for tid in range(THREADS):
        for m in range(E):
            out[line_of(tid), pos_load(tid, m)] = v[tid, m]
    return mid, out


def main():
    assert len({lds_slot(p, l) for p in range(N) for l in range(2)}) == 2 * N
    # the state maps are bijections onto (line, position)
    for f in (pos_load, pos_b, pos_c, pos_d):
        s = {(line_of(t), f(t, m)) for t in range(THREADS) for m in range(E)}
        assert len(s) == 2 * N, f.__name__
    rng = np.random.default_rng(1)
    x = (rng.standard_normal((2, N)) + 1j * rng.standard_normal((2, N))).astype(np.complex64)
    for col_like in (True, False):
        mid, out = run_pair(x, col_like)
        ref_mid = np.fft.fft(x.astype(np.complex128)) if col_like else np.fft.ifft(x.astype(np.complex128)) * N
        e1 = np.abs(mid - ref_mid).max() / np.abs(ref_mid).max()
        e2 = np.abs(out / N - x).max() / np.abs(x).max()
        print(f"{'column (fwd, inv)' if col_like else 'row (inv, fwd)'}: middle rel err {e1:.2e}, round trip {e2:.2e}")
        assert e1 < 1e-5 and e2 < 1e-5
    print("X2 write (state B) extra cycles:", bank_conflicts(pos_b, "write"),
          " read (state C):", bank_conflicts(pos_c, "read"))
    print("X2^H write (state C):", bank_conflicts(pos_c, "write"), " read (state B):", bank_conflicts(pos_b, "read"))
    print("model ok")


if __name__ == "__main__":
    main()
