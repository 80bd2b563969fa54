"""numpy-stream initial phases on the device (csrc/phase_mt.hip) and the device int16 join
(csrc/wav_io.hip) against numpy itself.

The reference draws each sentence's Griffin-Lim phases with np.random.rand(*S.shape) from numpy's
global legacy MT19937 (utils/audio.py:183) and joins a request's sentences as a Python list into
save_wav's int16 conversion (server/synthesizer.py:157-161, utils/audio.py:56-58).  The oracle of
both is numpy: np.random.rand / np.random.get_state, and the reference's own list-join expression.
CPU: the block schedule the kernel runs (oracle/mt19937_oracle.py) against numpy.  GPU: the kernel,
the Griffin-Lim runs that use it, the int16 join, and Synthesizer.tts bytes against the host path.
"""
import io

import numpy as np
import pytest
import torch

from conftest import load_pkg
from oracle import mt19937_oracle as mto

# (seed, 32-bit words drawn before: odd counts leave an odd position, frames per sentence)
CASES = [
    (0, 0, [3, 1, 7]),            # fresh seed: position 624
    (1, 2, [2, 5]),
    (1234, 6, [40]),
    (9, 622, [13, 2, 300]),       # draws that straddle many blocks
    (5, 2, [0, 4, 0, 1]),         # empty sentences draw nothing
    (3, 1, [7, 622, 3]),          # odd position: pairs straddle block boundaries
    (11, 5, [1, 1, 1, 1, 1, 1]),
]


def _pre(seed, words):
    np.random.seed(seed)
    for _ in range(words % 2):
        np.random.randint(1000)  # one 32-bit word: an odd position
    np.random.rand(words // 2)


def _numpy_draws(F):
    return [np.random.rand(1025, f) for f in F]


@pytest.mark.parametrize("seed,words,F", CASES)
def test_block_schedule_matches_numpy(seed, words, F):
    _pre(seed, words)
    st = np.random.get_state()
    out, key, pos = mto.draw_phases(st[1], st[2], F)
    ref = _numpy_draws(F)
    st2 = np.random.get_state()
    for b, f in enumerate(F):
        assert np.array_equal(out[b, :, :f], ref[b]), b
    assert np.array_equal(key, st2[1]) and pos == st2[2]


def test_reference_list_join_equals_concatenate():
    """The join Synthesizer.tts builds (a Python list of floats and int zeros -> save_wav) is the
    float64 concatenation: the device join restates that array, so bytes can match."""
    rng = np.random.default_rng(3)
    ws = [rng.standard_normal(n) * 0.3 for n in (5, 0, 17)]
    wavs = []
    for w in ws:
        wavs += list(w)
        wavs += [0] * 10000
    a = np.array(wavs)
    b = np.concatenate([np.concatenate([w, np.zeros(10000)]) for w in ws])
    assert a.dtype == np.float64 and np.array_equal(a, b)


# ---------------------------------------------------------------- GPU
def _ap(cfg):
    return load_pkg("audio").AudioProcessor(**cfg)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,words,F", CASES)
def test_device_phases_match_numpy(audio_cfg, seed, words, F):
    ap = _ap(audio_cfg)
    _pre(seed, words)
    with ap.numpy_phases():
        got = ap.draw_phases(F, Fmax=max(F) + 3).cpu().numpy()
    st_dev = np.random.get_state()
    _pre(seed, words)
    ref = _numpy_draws(F)
    st_ref = np.random.get_state()
    for b, f in enumerate(F):
        assert np.array_equal(got[b, :, :f], ref[b]), b
        assert not got[b, :, f:].any()
    assert np.array_equal(st_dev[1], st_ref[1]) and st_dev[2] == st_ref[2]


@pytest.mark.gpu
def test_device_phases_long_sentence(audio_cfg):
    """A Synthesizer-cap sentence (3021 frames, ~6.2 M words, ~10 k block steps) and the next draw."""
    ap = _ap(audio_cfg)
    np.random.seed(2024)
    with ap.numpy_phases():
        got = ap.draw_phases([3021]).cpu().numpy()
    nxt = np.random.rand(4)
    np.random.seed(2024)
    ref = np.random.rand(1025, 3021)
    assert np.array_equal(got[0], ref)
    assert np.array_equal(nxt, np.random.rand(4))


@pytest.mark.gpu
def test_griffin_lim_numpy_phases_equal_host_draws(audio_cfg):
    """A Griffin-Lim batch under numpy_phases() is bitwise the run with the host-drawn
    np.random.rand(1025, F_b) phases uploaded (the pre-round-6 path), for the persistent (small)
    and batched (large) loops."""
    ap = _ap({**audio_cfg, "griffin_lim_iters": 4})
    rng = np.random.default_rng(1)
    for F in ([40], [30, 300, 77]):
        mel = torch.from_numpy(rng.uniform(0, 1, (len(F), max(F), 80)).astype(np.float32)).cuda()
        np.random.seed(42)
        with ap.numpy_phases():
            a = ap.griffin_lim_batch(mel, F).cpu().numpy()
        after = np.random.rand(3)
        np.random.seed(42)
        pu = np.zeros((len(F), 1025, max(F)))
        for b, f in enumerate(F):
            pu[b, :, :f] = np.random.rand(1025, f)
        b_ = ap.griffin_lim_batch(mel, F, phase_u=pu).cpu().numpy()
        assert np.array_equal(a, b_), F
        assert np.array_equal(after, np.random.rand(3))


@pytest.mark.gpu
@pytest.mark.parametrize("peak", [None, 0.75, 0.004])
def test_pcm16_join_matches_reference_expression(audio_cfg, peak):
    """tts_gl_save_pcm16 vs the reference's own arithmetic: list join with 10 000 zeros, then
    wav * (32767 / max(0.01, max|wav|)) -> astype(int16); exact values at the peak included."""
    ap = _ap(audio_cfg)
    rng = np.random.default_rng(7)
    lens = [1000, 0, 12345, 7]
    pitch = 13000
    w = rng.standard_normal((len(lens), pitch)) * 0.2
    w[2, 17] = 0.9  # the global peak, exactly representable scale edge
    w[0, 3] = -0.9
    if peak == 0.004:
        w *= 0.004  # below save_wav's 0.01 floor
    wd = torch.from_numpy(w).cuda()
    got = ap.pcm16_join(wd, lens, gap=10000, peak=None if peak == 0.004 else peak)
    wavs = []
    for b, n in enumerate(lens):
        wavs += list(w[b, :n])
        wavs += [0] * 10000
    wav = np.array(wavs)
    p = np.max(np.abs(wav)) if peak in (None, 0.004) else peak
    ref = (wav * (32767 / max(0.01, p))).astype(np.int16)
    assert got.dtype == np.int16 and np.array_equal(got, ref)


@pytest.mark.gpu
def test_synthesizer_tts_bytes_equal_host_path(audio_cfg):
    """Synthesizer.tts (device phases + device join) returns exactly the bytes of the host path it
    replaces: host np.random.rand phases per sentence in order, the decode + Griffin-Lim of the same
    model, the reference's list join and save_wav (1- and 2-sentence requests, serial one-call
    dispatch)."""
    import scipy.io.wavfile
    synth = load_pkg("synthesis")
    text = load_pkg("text")
    from test_gpu_batched import _t2
    cfg, m = _t2(max_batch=4)
    m.decoder.max_decoder_steps = 400
    a = {**audio_cfg, "griffin_lim_iters": 8}
    ap = _ap(a)
    adapter = lambda s: text.text_to_sequence(s, ["basic_cleaners"])  # noqa: E731
    s = synth.Synthesizer(m, ap, cfg, input_adapter=adapter)
    s.tts_model.decoder.max_decoder_steps = 400
    for txt in ("Then we left the house.", "It took me a long time. Then we left!"):
        np.random.seed(99)
        buf = s.tts(txt)
        after = np.random.rand(2)
        np.random.seed(99)
        wavs = []
        ids = [np.asarray(adapter(sen)) for sen in s.sentences(txt)]
        # the decode the Synthesizer dispatches (one resident batch call for 2+ sentences when the
        # batch decoder takes them, else per sentence): its fp32 order is not the thing under test
        if len(ids) > 1 and synth._resident_batch(m, ids):
            o = m.inference_batch(ids)
            F = o["frames"]
            pu = np.zeros((len(F), 1025, max(F)))
            for b, T in enumerate(F):
                pu[b, :, :T] = np.random.rand(1025, T)
            wb = ap.griffin_lim_batch(o["mel_post"][:, :max(F)].contiguous(), F, phase_u=pu)
            for b, T in enumerate(F):
                wavs += list(wb[b, :ap.hop_length * (T - 1)].cpu().numpy())
                wavs += [0] * 10000
        else:
            for x in ids:
                o = m.inference_batch([x])
                T = o["frames"][0]
                pu = np.random.rand(1025, T)[None]
                w = ap.griffin_lim_batch(o["mel_post"], [T], phase_u=pu)[0, :ap.hop_length * (T - 1)].cpu().numpy()
                wavs += list(w)
                wavs += [0] * 10000
        ref = io.BytesIO()
        ap.save_wav(np.array(wavs), ref)
        assert buf.getvalue() == ref.getvalue(), txt
        assert np.array_equal(after, np.random.rand(2))
