"""CPU model of gl_iter_wave_kernel's data movement (csrc/griffin_lim.hip): the one-wave-per-frame
1024-point FFT as radix 16 x 16 x 4 over 64 lanes x 16 registers, its two LDS all-to-alls per FFT
(real / imaginary rounds through the XOR-swizzled slots wv_a1 / wv_a2), the natural-order Z slots
wv_sig, the bin-pair phase step with the in-place partner exchange, and the LDS bank rules of
MI355X_MICROARCH.md (ds_write_b64: 16-lane contiguous groups over 32 banks; ds_read_b64: 32-lane
halves over 64 banks).  The kernel's index maps are restated here lane by lane (numpy complex128
for the arithmetic) and checked against numpy's FFT and against the reference GL step math
(librosa 0.6.2 stft -> complex64 -> unit phase x |S| -> istft frame), so a change to a slot map or
a register mapping that breaks the algorithm or introduces bank conflicts fails on the CPU."""
import numpy as np

NH = 1024
LN = np.arange(64)
P1 = LN & 3
K2 = LN >> 2


def wv_a1(k2, n1):
    return k2 * 64 + (n1 ^ (4 * (k2 & 7)))


def wv_a2(k2, p1, q2):
    return k2 * 64 + 4 * (q2 ^ (k2 & 7)) + (p1 ^ (k2 & 3))


def wv_sig(k):
    return k ^ (((k >> 4) & 3) << 2)


def dft(v, n, sign):
    idx = np.arange(n)
    return v @ np.exp(sign * 2j * np.pi * np.outer(idx, idx) / n)


def xchg(v, wslot, rslot):
    """wave_xchg: every lane stores register r at wslot(r) (its own lane-vector of slots), then
    reads register r from rslot(r); done as the kernel does it, real parts then imaginary parts."""
    out = np.zeros_like(v)
    for part in (np.real, np.imag):
        lds = np.full(NH + 1, np.nan)
        for r in range(16):
            slots = wslot(r)
            assert len(set(slots.tolist())) == 64  # no two lanes store to one slot
            lds[slots] = part(v[:, r])
        for r in range(16):
            vals = lds[rslot(r)]
            assert not np.isnan(vals).any()  # every slot read was stored this round
            out[:, r] += vals if part is np.real else 1j * vals
    return out


def wave_fft(v, sign):
    """wave_fft1024: in v[L][r] = z[L + 64 r]; out v[L][4 j + q1] = Z[256 q1 + 64 j + 16 (L&3) + (L>>2)]."""
    v = dft(v, 16, sign)
    v = v * np.exp(sign * 2j * np.pi * np.outer(LN, np.arange(16)) / 1024)  # w^k2, w = W1024^L
    v = xchg(v, lambda k2: wv_a1(k2, LN), lambda p2: wv_a1(K2, P1 + 4 * p2))
    v = dft(v, 16, sign)
    v = v * np.exp(sign * 2j * np.pi * np.outer(P1, np.arange(16)) / 64)  # t2[q2][p1] = W64^(p1 q2)
    v = xchg(v, lambda q2: wv_a2(K2, P1, q2), lambda r: wv_a2(K2, r & 3, 4 * (r >> 2) + P1))
    for j in range(4):
        v[:, 4 * j:4 * j + 4] = dft(v[:, 4 * j:4 * j + 4], 4, sign)
    return v


def out_index():
    idx = np.zeros((64, 16), int)
    for j in range(4):
        for q1 in range(4):
            idx[:, 4 * j + q1] = 256 * q1 + 64 * j + 16 * P1 + K2
    return idx


def test_wave_fft_matches_numpy_both_directions():
    rng = np.random.default_rng(0)
    z = rng.standard_normal(NH) + 1j * rng.standard_normal(NH)
    v = z[LN[:, None] + 64 * np.arange(16)[None, :]]
    idx = out_index()
    assert sorted(idx.ravel().tolist()) == list(range(NH))
    np.testing.assert_allclose(wave_fft(v, -1), np.fft.fft(z)[idx], atol=1e-9)
    np.testing.assert_allclose(wave_fft(v, +1), np.fft.ifft(z)[idx] * NH, atol=1e-9)


def test_slot_maps_are_permutations():
    assert sorted(wv_a1(k, n) for k in range(16) for n in range(64)) == list(range(NH))
    assert sorted(wv_a2(k, p, q) for k in range(16) for p in range(4) for q in range(16)) == list(range(NH))
    assert sorted(wv_sig(k) for k in range(NH)) == list(range(NH))
    # the bin-pair step addresses Z by one per-lane base + multiples of 64 slots (sig permutes
    # bits 2-3 by bits 4-5 only)
    k = np.arange(NH)
    assert np.all(wv_sig(k) - (k & ~63) == wv_sig(k & 63))


def _conflicts(addr, groups, banks):
    extra = 0
    for g in groups:
        seen = {}
        for L in g:
            a = int(addr[L]) * 8
            for d in range(2):
                seen.setdefault((a // 4 + d) % banks, set()).add(a // 4 + d)
        extra += max(len(s) for s in seen.values()) - 1
    return extra


W64 = [list(range(16 * i, 16 * i + 16)) for i in range(4)]  # ds_write_b64 lane groups
R64 = [list(range(0, 32)), list(range(32, 64))]  # ds_read_b64 lane groups


def test_exchanges_are_bank_conflict_free():
    r3 = P1
    assert sum(_conflicts(wv_a1(k, LN), W64, 32) for k in range(16)) == 0
    assert sum(_conflicts(wv_a1(K2, P1 + 4 * p2), R64, 64) for p2 in range(16)) == 0
    assert sum(_conflicts(wv_a2(K2, P1, q), W64, 32) for q in range(16)) == 0
    assert sum(_conflicts(wv_a2(K2, pp, 4 * j + r3), R64, 64) for j in range(4) for pp in range(4)) == 0
    zw = [wv_sig(256 * q1 + 64 * j + 16 * r3 + K2) for j in range(4) for q1 in range(4)]
    assert sum(_conflicts(a, W64, 32) for a in zw) == 0
    assert sum(_conflicts(wv_sig(LN + 64 * m), R64, 64) for m in range(16)) == 0
    # the partner reads / in-place stores: a few 2-way conflicts at lane 0's wrap (measured: 16+28
    # extra cycles over a frame's 16 instructions)
    assert sum(_conflicts(wv_sig((NH - LN - 64 * m) & (NH - 1)), R64, 64) for m in range(8)) <= 16
    assert sum(_conflicts(wv_sig(NH - LN - 64 * m), W64, 32) for m in range(1, 8)) <= 32


def test_bin_pair_step_matches_reference_gl_frame():
    """One GL iteration of one frame through the kernel's data flow vs the reference math:
    X = rfft(window * y) rounded to complex64, X' = |S| X / |X| (DC / Nyquist real), y' =
    irfft(X') -- with the kernel's bin pairs (k, 1024 - k), its partner exchange into the slot of
    Z[1024 - k] (lane 0, m = 0 into the spare slot 1024), and k = 512 on its own."""
    rng = np.random.default_rng(1)
    x = rng.standard_normal(2048)
    S = np.abs(rng.standard_normal(1025)) + 0.1
    tw = np.exp(-2j * np.pi * np.arange(2048) / 2048)
    z = x[0::2] + 1j * x[1::2]
    Zr = wave_fft(z[LN[:, None] + 64 * np.arange(16)[None, :]], -1)
    lds = np.zeros(NH + 1, complex)  # natural-order Z at wv_sig(k)
    lds[wv_sig(out_index())] = Zr

    def unit(X, s):
        X = complex(np.complex64(X))
        m2 = X.real ** 2 + X.imag ** 2
        return s * X / np.sqrt(m2) if m2 > 0 else complex(s, 0)

    def presplit2(xk, xm, t):  # 2 z'[k]
        E = xk + np.conj(xm)
        D = (xk - np.conj(xm)) * np.conj(t)
        return E + 1j * D

    zb = wv_sig(LN)
    mb = wv_sig((64 - LN) & 63) + np.where(LN == 0, 64, 0)
    v = np.zeros((64, 16), complex)
    for m in range(8):
        k = LN + 64 * m
        zk = lds[zb + 64 * m]
        zm = np.where(LN == 0, zk, lds[mb + 64 * (15 - m)]) if m == 0 else lds[mb + 64 * (15 - m)]
        E = zk + np.conj(zm)
        O = -1j * (zk - np.conj(zm))
        tO = O * tw[k]
        xk = np.array([unit(e, s) for e, s in zip(E + tO, S[k])])
        xm = np.array([unit(e, s) for e, s in zip(np.conj(E - tO), S[NH - k])])
        if m == 0:
            xk[0] = xk[0].real
            xm[0] = xm[0].real
        v[:, m] = presplit2(xk, xm, tw[k])
        lds[mb + 64 * (15 - m)] = presplit2(xm, xk, -np.conj(tw[k]))  # in place (lane 0, m 0: slot 1024)
    z512 = lds[512]
    x512 = unit(2 * z512.real + 2 * z512.imag * tw[512], S[512])
    lds[512] = presplit2(x512, x512, tw[512])
    for R in range(8, 16):
        v[:, R] = lds[zb + 64 * R]
    zo = np.zeros(NH, complex)
    zo[out_index()] = wave_fft(v, +1)
    got = np.empty(2048)
    got[0::2] = zo.real * (0.5 / NH)
    got[1::2] = zo.imag * (0.5 / NH)

    X = np.fft.rfft(x).astype(np.complex64).astype(np.complex128)
    Xp = np.array([unit(X[k], S[k]) for k in range(1025)])
    Xp[0] = Xp[0].real
    Xp[1024] = Xp[1024].real
    ref = np.fft.irfft(Xp, 2048)
    np.testing.assert_allclose(got, ref, atol=1e-12 * np.abs(ref).max())


def test_chebyshev_window_recurrence():
    """The periodic Hann by c_{r+1} = 2 cos(theta) c_r - c_{r-1} over the lanes' 16 samples (step 128),
    from the host's two seeds per lane and parity: within 1e-14 of the window table."""
    win, woff = 1102, (2048 - 1102) // 2
    n = np.arange(2048) - woff
    table = np.where((n >= 0) & (n < win), 0.5 - 0.5 * np.cos(2 * np.pi * n / win), 0.0)
    K = 2 * np.cos(2 * np.pi * 128 / win)
    for e in (0, 1):
        s = 2 * LN + e
        a = 2 * np.pi * (s - woff) / win
        c0, c1 = np.cos(a), np.cos(a + 2 * np.pi * 128 / win)
        for r in range(16):
            sr = s + 128 * r
            ins = (sr >= woff) & (sr < woff + win)
            w = 0.5 - 0.5 * c0
            np.testing.assert_allclose(w[ins], table[sr[ins]], atol=1e-14)
            c0, c1 = c1, K * c1 - c0
