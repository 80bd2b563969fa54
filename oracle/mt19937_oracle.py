"""TEST INFRASTRUCTURE ONLY (never imported by the product path): a numpy restatement of the
block schedule of ``your-voice-tts_amd/csrc/phase_mt.hip`` (the device continuation of numpy's
legacy MT19937 stream), checked in ``tests/test_phase_mt.py`` against numpy itself.

What it restates: ``np.random.rand(1025, F_b)`` for b = 0..B-1 in order (the reference's
``_griffin_lim`` phases, utils/audio.py:183, one draw per sentence as server/synthesizer.py:145-158
synthesises them) from a legacy ``np.random.get_state()`` state, and the state numpy holds after
those draws.  numpy's MT19937 (numpy/random/src/mt19937/mt19937.c, legacy RandomState):
``mt19937_gen`` twists the 624-word key in place, ``mt19937_next`` tempers ``key[pos++]``, and
``random_sample`` = ``mt19937_next_double`` = ((w0 >> 5) * 2^26 + (w1 >> 6)) / 2^53.  Parity is
pinned by numpy itself (the oracle of this test is ``np.random.rand``).
"""
from __future__ import annotations

import numpy as np

N, M, K = 624, 397, 227
NB = 1025


def _mix(a, b):
    y = (a & np.uint32(0x80000000)) | (b & np.uint32(0x7FFFFFFF))
    return (y >> np.uint32(1)) ^ np.where(y & np.uint32(1), np.uint32(0x9908B0DF), np.uint32(0))


def _temper(y):
    y = y ^ (y >> np.uint32(11))
    y = y ^ ((y << np.uint32(7)) & np.uint32(0x9D2C5680))
    y = y ^ ((y << np.uint32(15)) & np.uint32(0xEFC60000))
    return y ^ (y >> np.uint32(18))


def next_block(o):
    """The kernel's block step: thread t < 227 computes words t, t + 227, t + 454 (t <= 169) of the
    next block from the previous one; word 623 needs the new word 0 (recomputed)."""
    o = o.astype(np.uint32)
    n = np.empty(N, np.uint32)
    t = np.arange(K)
    x0 = o[t + M] ^ _mix(o[t], o[t + 1])
    x1 = x0 ^ _mix(o[t + K], o[t + K + 1])
    n[t] = x0
    n[t + K] = x1
    t2 = np.arange(N - 2 * K)  # 0..169
    i2 = t2 + 2 * K
    nxt = np.where(i2 < N - 1, o[np.minimum(i2 + 1, N - 1)], o[M] ^ _mix(o[0], o[1]))
    n[i2] = x1[t2] ^ _mix(o[i2], nxt)
    return n


def draw_phases(key, pos, F, Fmax=None):
    """Block-schedule restatement: returns (out [B][1025][Fmax] float64, key', pos')."""
    F = [int(f) for f in F]
    Fmax = max(F) if Fmax is None else Fmax
    B = len(F)
    out = np.zeros((B, NB, Fmax))
    off = np.concatenate([[0], np.cumsum([NB * f for f in F])]).astype(np.int64)
    D = int(off[-1])
    key = np.asarray(key, np.uint32)
    if D == 0:
        return out, key.copy(), int(pos)
    e = pos + 2 * D
    Kb = (e - 1) // N
    blocks = {0: key.copy()}

    def emit(kb):
        base = kb * N
        jlo = base - pos - 1
        jlo = 0 if jlo <= 0 else (jlo + 1) // 2
        hi = base + N - 2 - pos
        if hi < 0:
            return
        jhi = min(hi // 2, D - 1)
        if jhi < jlo:
            return
        j = np.arange(jlo, jhi + 1, dtype=np.int64)
        r0 = pos + 2 * j - base
        cur, prv = blocks[kb], blocks.get(kb - 1)
        w0 = np.where(r0 < 0, prv[N - 1] if prv is not None else 0, cur[np.maximum(r0, 0)]).astype(np.uint32)
        w1 = cur[r0 + 1]
        u = ((_temper(w0) >> np.uint32(5)).astype(np.float64) * 67108864.0 +
             (_temper(w1) >> np.uint32(6)).astype(np.float64)) * (1.0 / 9007199254740992.0)
        b = np.searchsorted(off, j, side="right") - 1
        local = j - off[b]
        fb = np.asarray(F)[b]
        k = local // fb
        f = local - k * fb
        out[b, k, f] = u

    emit(0)
    for kb in range(Kb):
        blocks[kb + 1] = next_block(blocks[kb])
        blocks.pop(kb - 1, None)
        emit(kb + 1)
    return out, blocks[Kb].copy(), int(e - Kb * N)
