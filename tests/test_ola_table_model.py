"""CPU model of gl_ola_kernel's window sum-square table (csrc/griffin_lim.hip): for a sample whose
contributing frames all exist, librosa istft's float32 window sum-square (win^2 of frames
ilo..ihi added in frame order, each addition rounded to float32) depends only on
(q - woff) mod hop, so the kernel reads it from a [hop] table the host sums once.  Checked here
sample by sample against the direct sum (ola_sample's loop), for the reference geometry and
others, including where the kernel must fall back to the direct sum (clipped contributors)."""
import numpy as np
import pytest

NFFT = 2048


def geometry(win):
    woff = (NFFT - win) // 2
    n = np.arange(win)
    w = 0.5 - 0.5 * np.cos(2 * np.pi * n / win)
    win2 = np.zeros(NFFT)
    win2[woff:woff + win] = w * w
    return woff, win2


def direct(q, F, hop, win, woff, win2):
    """ola_sample's window sum-square loop."""
    if q < woff:
        return np.float32(0), False
    u = q - woff
    raw = u - win + 1
    ilo = 0 if raw <= 0 else (raw + hop - 1) // hop
    ihi = min(u // hop, F - 1)
    wss = np.float32(0)
    for i in range(ilo, ihi + 1):
        wss = np.float32(np.float64(wss) + win2[q - i * hop])
    return wss, raw >= 1 and u // hop <= F - 1


def table(hop, win, woff, win2):
    """The host's [hop] table (tts_gl_create)."""
    t = np.zeros(hop, np.float32)
    for r in range(hop):
        u = r + hop * (win // hop + 1)
        ilo, ihi = (u - win + 1 + hop - 1) // hop, u // hop
        w = np.float32(0)
        for i in range(ilo, ihi + 1):
            w = np.float32(np.float64(w) + win2[woff + u - i * hop])
        t[r] = w
    return t


@pytest.mark.parametrize("hop,win,F", [(275, 1102, 40), (256, 1024, 30), (200, 800, 25), (300, 2048, 20),
                                       (275, 275, 12), (1, 7, 9)])
def test_window_sum_square_table_matches_direct_sum(hop, win, F):
    woff, win2 = geometry(win)
    t = table(hop, win, woff, win2)
    N = hop * (F - 1)
    n_full = 0
    for p in range(N):
        q = p + NFFT // 2
        ref, full = direct(q, F, hop, win, woff, win2)
        if full:
            n_full += 1
            assert t[(q - woff) % hop] == ref, (p, q)
    assert n_full > 0
