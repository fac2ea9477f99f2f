#!/usr/bin/env python3
"""NumPy model of a wave-shuffle transform pair for 4096-point rows (one row
per 256-thread workgroup, 16 complex slots per thread, radices 16.16.16), the
4096 counterpart of tools/shuffle_fft_model.py:

  A (load/store)  slots pos 8-11   lanes l0..l5 = pos 0-5        waves = pos 6, 7
  P1 radix 16, twiddle w_4096^(t k1)
  X1 LDS (+ barrier)
  B               slots pos 4-7    l1, l3, l4, l5 = pos 0-3   l0, l2, w0, w1 = pos 8-11
  P2 radix 16, twiddle w_256^(n k2), n = pos 0-3
  X2 registers:   slot bit 0 <-> l1 (quad_perm xor 2), bit 1 <-> l3 (row_ror:8 with
                  bank masks), bit 2 <-> l4 (v_permlane16_swap), bit 3 <-> l5
                  (v_permlane32_swap)
  C               slots pos 0-3    l1, l3, l4, l5 = pos 4-7
  P3 radix 16; slot m then holds frequency klow(tid) + 256 m.

Checks the pair against numpy.fft and searches the X1 LDS swizzle for zero
bank conflicts in both directions. python tools/shuffle4096_model.py
"""
import itertools

import numpy as np

N, E, THREADS = 4096, 16, 256


def bit(x, i):
    return (x >> i) & 1


def lanes(tid):
    lam = tid & 63
    return [bit(lam, i) for i in range(6)], [bit(tid >> 6, 0), bit(tid >> 6, 1)]


def pos_a(tid, m):
    return tid | (m << 8)


def pos_b(tid, m):
    l, w = lanes(tid)
    p = (l[1] << 0) | (l[3] << 1) | (l[4] << 2) | (l[5] << 3)
    p |= m << 4
    p |= (l[0] << 8) | (l[2] << 9) | (w[0] << 10) | (w[1] << 11)
    return p


def pos_c(tid, m):
    l, w = lanes(tid)
    p = m
    p |= (l[1] << 4) | (l[3] << 5) | (l[4] << 6) | (l[5] << 7)
    p |= (l[0] << 8) | (l[2] << 9) | (w[0] << 10) | (w[1] << 11)
    return p


def klow(tid):
    l, w = lanes(tid)
    return l[0] | (l[2] << 1) | (w[0] << 2) | (w[1] << 3) | (l[1] << 4) | (l[3] << 5) | (l[4] << 6) | (l[5] << 7)


def partner_swap(v, sbit, lbit):
    """slot bit sbit <-> lane bit lbit, by whatever instruction (semantics only)"""
    out = v.copy()
    for tid in range(THREADS):
        x = bit(tid, lbit)
        for m in range(E):
            y = bit(m, sbit)
            # after: lane bit = old slot bit, slot bit = old lane bit
            src_tid = (tid & ~(1 << lbit)) | (y << lbit)
            src_m = (m & ~(1 << sbit)) | (x << sbit)
            out[tid, m] = v[src_tid, src_m]
    return out


def x2(v):
    for sbit, lbit in ((0, 1), (1, 3), (2, 4), (3, 5)):
        v = partner_swap(v, sbit, lbit)
    return v


def dft(u, inv):
    k = np.arange(len(u))
    return np.exp((2j if inv else -2j) * np.pi * np.outer(k, k) / len(u)) @ u


def root(e, inv):
    z = np.exp(-2j * np.pi * (e % N) / N).astype(np.complex64)
    return np.conj(z) if inv else z


def tw(tid, kind):
    if kind == 1:
        return [tid * k for k in range(1, 16)]
    if kind == 2:
        l, _ = lanes(tid)
        n = l[1] | (l[3] << 1) | (l[4] << 2) | (l[5] << 3)
        return [16 * n * k for k in range(1, 16)]
    return None


def dpass(v, kind, inv, dif):
    for tid in range(THREADS):
        u = v[tid].astype(np.complex128)
        t = tw(tid, kind)
        if t is not None and not dif:
            u[1:] *= [root(e, inv) for e in t]
        u = dft(u, inv)
        if t is not None and dif:
            u[1:] *= [root(e, inv) for e in t]
        v[tid] = u.astype(np.complex64)


def make_slot(h_of):
    def slot(p):
        return p ^ h_of(p >> 8)
    return slot


def lds(v, src, dst, slot):
    mem = {}
    for tid in range(THREADS):
        for m in range(E):
            mem[slot(src(tid, m))] = v[tid, m]
    out = np.empty_like(v)
    for tid in range(THREADS):
        for m in range(E):
            out[tid, m] = mem[slot(dst(tid, m))]
    return out


def conflicts(pos_fn, slot, kind):
    total = 0
    grp, nb = (32, 64) if kind == "read" else (16, 32)
    for w in range(THREADS // 64):
        for m in range(E):
            addr = [2 * slot(pos_fn(t, m)) for t in range(w * 64, w * 64 + 64)]
            for g0 in range(0, 64, grp):
                banks = {}
                for a in addr[g0:g0 + grp]:
                    for d in (a, a + 1):
                        banks.setdefault(d % nb, set()).add(d)
                total += max(len(x) for x in banks.values()) - 1
    return total


def all_conflicts(slot):
    return (conflicts(pos_a, slot, "write"), conflicts(pos_b, slot, "read"),
            conflicts(pos_b, slot, "write"), conflicts(pos_a, slot, "read"))


def main():
    for f in (pos_a, pos_b, pos_c):
        assert len({f(t, m) for t in range(THREADS) for m in range(E)}) == N
    assert sorted(klow(t) for t in range(THREADS)) == list(range(256))
    # X1 slot swizzle: p ^ H(j), j = p >> 8; H puts j0 on bit 3 and j1 on bits
    # 2 and 4: B-side 16-lane writes see (pos0, pos1, j1, j0) on bits 0-3, B-side
    # 32-lane reads a bijection of (pos0, pos1, pos2, j0, j1) onto bits 0-4
    def h(j):
        return (bit(j, 0) << 3) | (bit(j, 1) << 2) | (bit(j, 1) << 4)
    slot = make_slot(h)
    c = all_conflicts(slot)
    print("X1 swizzle conflicts A-write/B-read/B-write/A-read:", c)
    assert len({slot(p) for p in range(N)}) == N
    rng = np.random.default_rng(3)
    x = (rng.standard_normal(N) + 1j * rng.standard_normal(N)).astype(np.complex64)
    v = np.array([[x[pos_a(t, m)] for m in range(E)] for t in range(THREADS)], np.complex64)
    inv1 = True  # row pass: inverse, then forward
    dpass(v, 1, inv1, True)
    v = lds(v, pos_a, pos_b, slot)
    dpass(v, 2, inv1, True)
    v = x2(v)
    dpass(v, 3, inv1, True)
    mid = np.empty(N, np.complex64)
    for t in range(THREADS):
        for m in range(E):
            mid[klow(t) + 256 * m] = v[t, m]
    ref = np.fft.ifft(x.astype(np.complex128)) * N
    e1 = np.abs(mid - ref).max() / np.abs(ref).max()
    dpass(v, 3, False, False)
    v = x2(v)
    dpass(v, 2, False, False)
    v = lds(v, pos_b, pos_a, slot)
    dpass(v, 1, False, False)
    out = np.array([v[t, m] for m in range(E) for t in range(THREADS)])  # index t + 256 m
    e2 = np.abs(out / N - x).max() / np.abs(x).max()
    print(f"middle rel err {e1:.2e}, round trip {e2:.2e}")
    assert e1 < 1e-5 and e2 < 1e-5 and sum(c) == 0
    print("model ok")


if __name__ == "__main__":
    main()
