#!/usr/bin/env python3
"""Host model of the index arithmetic of k_rows_xp (N = 16384, 64 x 256 split), k_rows_hp (N = 4096,
16 x 256 split) and k_cols_half HX (N = 4096, 16 x 16 x 16): the LDS slots of T_in / T_out, the in-wave register <-> lane bit transpositions of
device/lane_xchg.h (element (R = r, L = l) -> (R = l, L = r)), the twiddles and the output layout,
played on numpy arrays [thread][register] and checked against N * ifft (the unnormalised inverse
transform, sign +). It validates the kernels' indexing on the CPU; the hardware semantics of the
permlane / DPP swaps are checked on the GPU by tools/microbench/rm16bench (lane_xchg check).
Usage: python tools/xp_model.py"""
import numpy as np

RS = 260  # k_rows_xp
RS_HP = 264  # k_rows_hp


def slot(n1, j):
    return n1 * RS + (j ^ ((n1 >> 2) & 3))


def hp_swz(n1):
    return ((n1 >> 1) & 7) ^ (((n1 >> 1) & 1) << 2)


def slot_hp(n1, j):
    return n1 * RS_HP + (j ^ hp_swz(n1))


def W(e, n):
    return np.exp(2j * np.pi * e / n)


def idft(v, axis):
    """X[k] = sum_n x[n] exp(+2 pi i n k / r) along `axis`"""
    r = v.shape[axis]
    return np.fft.ifft(v, axis=axis) * r


def swap_reg_lane(v, rb, lb):
    """v[t, m]; swap register bit rb with lane bit lb of t (t = wave * 64 + lane)"""
    out = np.empty_like(v)
    T, M = v.shape
    for t in range(T):
        for m in range(M):
            r_bit, l_bit = (m >> rb) & 1, (t >> lb) & 1
            t2 = (t & ~(1 << lb)) | (r_bit << lb)
            m2 = (m & ~(1 << rb)) | (l_bit << rb)
            out[t2, m2] = v[t, m]
    return out


def fill_tin(x, N, T, sub_bits, slot=slot):
    """T_in writes as the kernels do (own lanes at i + m T, mirror lanes at N - i - m T, thread 0's
    m = 0 mirror at N/2) and checks every slot holds x(n) at slot(n mod 2^sub_bits, n >> sub_bits)"""
    nsub = 1 << sub_bits
    lds = {}
    for i in range(T):
        wo = slot(i & (nsub - 1), i >> sub_bits)
        nm = N - i
        wm = slot(nm & (nsub - 1), nm >> sub_bits)
        wm0 = slot(0, (N // 2) >> sub_bits) if i == 0 else wm
        step = T >> sub_bits
        for m in range(8):
            a = wo + step * m
            n = i + m * T
            assert a == slot(n & (nsub - 1), n >> sub_bits)
            assert a not in lds
            lds[a] = x[n]
            b = (wm0 if m == 0 else wm) - step * m
            n = N // 2 if (m == 0 and i == 0) else N - i - m * T
            assert b == slot(n & (nsub - 1), n >> sub_bits), (i, m)
            assert b not in lds
            lds[b] = x[n]
    assert len(lds) == N
    return lds


def model_xp(seed=1):
    N, T = 16384, 1024
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    lds = fill_tin(x, N, T, 6)
    v = np.zeros((T, 16), complex)
    tid = np.arange(T)
    w, l = tid >> 6, tid & 63
    s, p = l & 3, l >> 2
    n1r = 4 * w + s
    rd = n1r * RS + (p ^ (w & 3))
    for t in range(T):
        for m in range(16):
            v[t, m] = lds[rd[t] + 16 * m]
    v = idft(v, 1)
    v *= W(64 * p[:, None] * np.arange(16)[None, :], N)
    for rb in range(4):
        v = swap_reg_lane(v, rb, rb + 2)
    v = idft(v, 1)
    v *= W(n1r[:, None] * (p[:, None] + 16 * np.arange(16)[None, :]), N)
    lds2 = {}
    for t in range(T):
        for m in range(16):
            lds2[rd[t] + 16 * m] = v[t, m]
    q, k2 = (tid >> 4) & 3, (tid & 15) + 16 * w
    for t in range(T):
        for r in range(16):
            v[t, r] = lds2[(q[t] + 4 * r) * RS + (k2[t] ^ (r & 3))]
    v = idft(v, 1)
    v *= W(256 * q[:, None] * np.arange(16)[None, :], N)
    v = swap_reg_lane(v, 2, 4)
    v = swap_reg_lane(v, 3, 5)
    out = v.copy()
    for c in range(4):
        grp = v[:, [c, c + 4, c + 8, c + 12]]
        out[:, [c, c + 4, c + 8, c + 12]] = idft(grp, 1)
    X = np.zeros(N, complex)
    for t in range(T):
        for m in range(16):
            X[k2[t] + 256 * (m & 3) + 1024 * q[t] + 4096 * (m >> 2)] = out[t, m]
    ref = np.fft.ifft(x) * N
    return np.max(np.abs(X - ref)) / np.max(np.abs(ref))


def model_hp(seed=2):
    N, T = 4096, 256
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    lds = fill_tin(x, N, T, 4, slot_hp)
    v = np.zeros((T, 16), complex)
    tid = np.arange(T)
    w, l = tid >> 6, tid & 63
    s, p = l & 3, l >> 2
    n1r = 4 * w + s
    rd = n1r * RS_HP + (p ^ hp_swz(n1r))
    for t in range(T):
        for m in range(16):
            v[t, m] = lds[rd[t] + 16 * m]
    v = idft(v, 1)
    v *= W(16 * p[:, None] * np.arange(16)[None, :], N)
    for rb in range(4):
        v = swap_reg_lane(v, rb, rb + 2)
    v = idft(v, 1)
    v *= W(n1r[:, None] * (p[:, None] + 16 * np.arange(16)[None, :]), N)
    lds2 = {}
    for t in range(T):
        for m in range(16):
            lds2[rd[t] + 16 * m] = v[t, m]
    for t in range(T):
        for n1 in range(16):
            v[t, n1] = lds2[n1 * RS_HP + (t ^ hp_swz(n1))]
    v = idft(v, 1)
    X = np.zeros(N, complex)
    for t in range(T):
        for m in range(16):
            X[t + 256 * m] = v[t, m]
    ref = np.fft.ifft(x) * N
    return np.max(np.abs(X - ref)) / np.max(np.abs(ref))


def model_hx(seed=3):
    """k_cols_half HX (fft_cols_hx): one 4096-point column, threads (w, a) with x(a + 16 w + 256 m) in
    v[m]; DFT over m, x W_N^((a + 16 w) k0), LDS transposition (register k0 <-> wave w), DFT over w,
    x W_256^(a k1), register <-> lane-bits-2..5 transposition (k1 <-> a), DFT over a: thread (w, a)
    then holds X(w + 16 a + 256 m). Also checks HX 2's storage-row permutation is a bijection."""
    N = 4096
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    w, a, m = np.meshgrid(np.arange(16), np.arange(16), np.arange(16), indexing="ij")
    v = x[a + 16 * w + 256 * m]              # v[w, a, m]
    v = idft(v, 2)
    v = v * W((a + 16 * w) * m, N)           # m now indexes k0
    v = np.transpose(v, (2, 1, 0))           # wave k0, lane a, register w
    v = idft(v, 2)                           # register k1
    v = v * W(16 * a * m, N)
    v = np.transpose(v, (0, 2, 1))           # lane k1, register a
    v = idft(v, 2)                           # register k2
    X = np.zeros(N, complex)
    X[w + 16 * a + 256 * m] = v
    ref = np.fft.ifft(x) * N
    store = lambda y: ((y & 15) << 8) | ((y >> 8) << 4) | ((y >> 4) & 15)  # noqa: E731
    back = lambda s: (s >> 8) | ((s & 15) << 4) | (((s >> 4) & 15) << 8)  # noqa: E731
    y = np.arange(N)
    assert np.array_equal(back(store(y)), y) and len(set(store(y).tolist())) == N
    # a store instruction (wave k0, register k2) covers 16 consecutive storage rows
    assert all(sorted(store(k0 + 16 * np.arange(16) + 256 * k2)) == list(range(256 * k0 + 16 * k2, 256 * k0 + 16 * k2 + 16))
               for k0 in range(16) for k2 in range(16))
    return np.max(np.abs(X - ref)) / np.max(np.abs(ref))


def hp_bank_multiplicity():
    """Worst bank multiplicity of k_rows_hp's four LDS access shapes (MI355X_MICROARCH.md §LDS:
    ds_write_b64 in 16-lane groups, bank of 8-B slot mod 16; ds_read_b64 in 32-lane groups, mod 32):
    T_in writes (16 consecutive n1, one j), T_in reads (lanes s + 4 p: n1 = 4 w + s, j = p + 16 m),
    T_out writes (the same slots, 16-lane groups), T_out reads (32 consecutive j, one n1). 1 = conflict-free."""
    def mult(v):
        return max(v.count(a) for a in v)
    w1 = max(mult([slot_hp(t, j) % 16 for t in range(16)]) for j in range(256))
    r1 = max(mult([slot_hp(4 * w + s, p + 8 * hh + 16 * m) % 32 for p in range(8) for s in range(4)])
             for w in range(4) for m in range(16) for hh in range(2))
    w2 = max(mult([slot_hp(4 * w + s, p + 4 * q + 16 * m) % 16 for p in range(4) for s in range(4)])
             for w in range(4) for m in range(16) for q in range(4))
    r2 = max(mult([slot_hp(n1, k0 + k) % 32 for k in range(32)]) for n1 in range(16) for k0 in range(0, 256, 32))
    return max(w1, r1, w2, r2)


if __name__ == "__main__":
    print(f"k_rows_hp LDS bank multiplicity (1 = conflict-free): {hp_bank_multiplicity()}")
    print(f"k_rows_xp model (16384): max |X - N ifft(x)| / max = {model_xp():.2e}")
    print(f"k_rows_hp model (4096):  max |X - N ifft(x)| / max = {model_hp():.2e}")
    print(f"k_cols_half HX model:    max |X - N ifft(x)| / max = {model_hx():.2e}")
