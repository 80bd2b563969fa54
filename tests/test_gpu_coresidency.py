"""Persistent kernels (resident decoder, resident encoder BiLSTM, persistent Griffin-Lim) hand data
between workgroups inside one launch, so they are only launched when every workgroup can be
resident at once (csrc/runtime.hip: launch_persistent — occupancy check, then a plain launch; TTS_COOP=1 for a cooperative one).
TTS_CU_CAP pretends the device has fewer CUs: the grids then cannot be co-resident, nothing
persistent is launched, and each stage must take its multi-launch fallback with unchanged results.
A persistent Griffin-Lim whose hand-off wait times out (fault injection) must raise and must not
hand out a plausible waveform."""
import os

import numpy as np
import pytest
import torch

from conftest import golden, golden_flags, load_pkg

pytestmark = pytest.mark.gpu


class _env:
    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update({k: str(v) for k, v in self.kv.items()})

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _t2():
    t2 = load_pkg("tacotron2")
    fl = golden_flags(golden("t2_fwdmask_L100"))
    m = t2.Tacotron2(130, 0, r=1, attn_win=fl["attn_win"], attn_norm=fl["attn_norm"], forward_attn=fl["forward_attn"],
                     trans_agent=fl["trans_agent"], forward_attn_mask=fl["forward_attn_mask"],
                     location_attn=fl["location_attn"], max_batch=4)
    return m.cuda().eval()


def test_persistent_griffin_lim_fallback_is_bitwise(audio_cfg):
    audio = load_pkg("audio")
    ap = audio.AudioProcessor(**{**audio_cfg, "griffin_lim_iters": 12})
    rng = np.random.Generator(np.random.PCG64(3))
    mel = torch.from_numpy(rng.uniform(0, 1, size=(1, 90, 80)).astype(np.float32)).cuda()
    pu = rng.uniform(0, 1, size=(1, 1025, 90))
    a = ap.griffin_lim_batch(mel, [90], phase_u=pu)
    assert ap.last_gl_path() == "persistent"
    with _env(TTS_CU_CAP=8):
        b = ap.griffin_lim_batch(mel, [90], phase_u=pu)
        assert ap.last_gl_path() == "fused"
    assert torch.equal(a, b)
    c = ap.griffin_lim_batch(mel, [90], phase_u=pu)  # and back
    assert ap.last_gl_path() == "persistent" and torch.equal(a, c)


def test_resident_decoder_and_encoder_fallback_match_multilaunch():
    z = golden("t2_fwdmask_L100")
    ids = [z["ids"]]
    m = _t2()
    ref = m.inference_batch(ids)
    assert m.last_timing["resident"] and m.last_timing["encoder_resident"]
    with _env(TTS_RESIDENT=0):
        ml = _t2()
        want = ml.inference_batch(ids)
        assert not ml.last_timing["resident"] and not ml.last_timing["encoder_resident"]
    with _env(TTS_CU_CAP=8):  # (the encoder's 128-thread workgroups fit 256 on 64 CUs)
        fb = _t2()
        got = fb.inference_batch(ids)
        assert not fb.last_timing["resident"] and not fb.last_timing["encoder_resident"]
    # the fallback IS the multi-launch path: bitwise equal to it
    for k in ("mel", "mel_post", "align", "stop"):
        assert torch.equal(got[k], want[k]), k
    assert got["frames"] == ref["frames"] == [z["mel"].shape[0]]
    # ... and within the parity tolerance of the resident path
    d = (got["mel_post"] - ref["mel_post"]).norm() / ref["mel_post"].norm()
    assert float(d) < 1e-5


def test_persistent_griffin_lim_timeout_raises_and_poisons(audio_cfg):
    """Fault injection: frame 3 of sentence 0 stops publishing after its first iteration, so its
    neighbours' hand-off waits time out.  The run must report an error and its waveform must be
    NaN (never a plausible signal); the same handle then works again."""
    audio = load_pkg("audio")
    with _env(TTS_GL_WAIT_TICKS=20000):  # 0.2 ms per wait at the 100 MHz wall clock
        ap = audio.AudioProcessor(**{**audio_cfg, "griffin_lim_iters": 8})
        rng = np.random.Generator(np.random.PCG64(4))
        mel = torch.from_numpy(rng.uniform(0, 1, size=(1, 40, 80)).astype(np.float32)).cuda()
        pu = rng.uniform(0, 1, size=(1, 1025, 40))
        good = ap.griffin_lim_batch(mel, [40], phase_u=pu)
        assert ap.last_gl_path() == "persistent" and torch.isfinite(good).all()
        with _env(TTS_GL_INJECT_DROP=3):
            with pytest.raises(RuntimeError, match="timed out"):
                ap.griffin_lim_batch(mel, [40], phase_u=pu)
        again = ap.griffin_lim_batch(mel, [40], phase_u=pu)
        assert torch.equal(again, good)


def test_synthesize_native_timeout_surfaces(audio_cfg):
    """The same fault through tts_synth_run: sync=True raises for the failing call itself; with
    sync=False the waveform is NaN and the next call raises."""
    audio = load_pkg("audio")
    z = golden("t2_fwdmask_L12")
    m = _t2()
    with _env(TTS_GL_WAIT_TICKS=20000):
        ap = audio.AudioProcessor(**{**audio_cfg, "griffin_lim_iters": 6})
        with _env(TTS_GL_INJECT_DROP=2):
            with pytest.raises(RuntimeError, match="timed out"):
                m.synthesize_native([z["ids"]], ap, seed=1, sync=True)
            wav, _ = m.synthesize_native([z["ids"]], ap, seed=1, sync=False)
            assert torch.isnan(wav).all()
        with pytest.raises(RuntimeError, match="timed out"):
            m.synthesize_native([z["ids"]], ap, seed=1, sync=True)
        wav, _ = m.synthesize_native([z["ids"]], ap, seed=1, sync=True)
        assert torch.isfinite(wav).all()


def test_long_sentence_after_griffin_lim_timeout(audio_cfg):
    """after a persistent Griffin-Lim timeout, a batch-1 sentence above 256 frames (its
    speculative Griffin-Lim in the decoder hook becomes an empty run, then the host redoes it) must
    not report the earlier run's failure: the empty run clears the status word too.  Its waveform
    equals the same sentence on a fresh handle."""
    audio = load_pkg("audio")
    z = golden("t2_fwdmask_L12")
    ids_long = load_pkg("weights").synthetic_ids(130, 7)  # 2L + 22 = 282 frames under the mask
    m = _t2()
    with _env(TTS_GL_WAIT_TICKS=20000):
        ap = audio.AudioProcessor(**{**audio_cfg, "griffin_lim_iters": 6})
        with _env(TTS_GL_INJECT_DROP=2):
            with pytest.raises(RuntimeError, match="timed out"):
                m.synthesize_native([z["ids"]], ap, seed=1, sync=True)
        wav, frames = m.synthesize_native([ids_long], ap, seed=1, sync=True)
        assert frames[0] > 256 and torch.isfinite(wav).all()
        ref, _ = _t2().synthesize_native([ids_long], ap, seed=1, sync=True)
    assert torch.equal(wav, ref)


def test_resident_decoder_timeout_reruns_multilaunch():
    """Fault injection: every hand-off wait of the resident decoder times out at once
    (TTS_DEC_WAIT_TICKS=1), as when a workgroup cannot become resident beside another stream's work.
    The call must not fail: the sentence re-runs from its initial state on the multi-launch path,
    bitwise that path's output; the next call on a normal handle is resident again."""
    z = golden("t2_fwdmask_L100")
    L = len(z["ids"])
    enc = _t2().encode(torch.from_numpy(z["ids"]).view(1, -1).cuda(), [L])  # one encoder output for all
    with _env(TTS_RESIDENT=0):
        want = _t2().inference_batch(None, enc=enc, lens=[L])
    with _env(TTS_DEC_WAIT_TICKS=1):
        m = _t2()
        got = m.inference_batch(None, enc=enc, lens=[L])
        assert not m.last_timing["resident"], "no timeout was injected"
    for k in ("mel", "mel_post", "align", "stop"):
        assert torch.equal(got[k], want[k]), k
    m2 = _t2()
    again = m2.inference_batch(None, enc=enc, lens=[L])
    assert m2.last_timing["resident"] and again["frames"] == want["frames"] == [z["mel"].shape[0]]


def test_batched_resident_encoder_matches_per_step_launches():
    """The batched resident BiLSTM (encoder_resident_batch_kernel: XCD-local hand-offs, MFMA gate
    rows) on a ragged 64-sentence batch against the per-step launches it replaces (TTS_CU_CAP makes
    the grid non-co-resident): same outputs within fp32 reduction-order noise, zero rows past each
    length; a second call takes the resident path again."""
    w = load_pkg("weights")
    lens = w.synthetic_lengths(64, 2)
    ids = torch.zeros(64, int(max(lens)), dtype=torch.long)
    for b, L in enumerate(lens):
        ids[b, :int(L)] = torch.from_numpy(w.synthetic_ids(int(L), 200 + b))
    m = _t2_batch(64)
    res = m.encode(ids.cuda(), [int(x) for x in lens])
    assert m._path_timing(*m._handles(ids.shape[1], 64)[:2])["encoder_path"] == 2
    with _env(TTS_CU_CAP=64):
        fb = _t2_batch(64)
        ref = fb.encode(ids.cuda(), [int(x) for x in lens])
        assert fb._path_timing(*fb._handles(ids.shape[1], 64)[:2])["encoder_path"] == 0
    for b, L in enumerate(lens):
        L = int(L)
        d = float((res[b, :L] - ref[b, :L]).norm() / ref[b, :L].norm())
        assert d < 1e-5, (b, d)
        assert torch.all(res[b, L:] == 0)
    again = m.encode(ids.cuda(), [int(x) for x in lens])
    assert torch.equal(again, res)  # deterministic


def _t2_batch(max_batch):
    t2 = load_pkg("tacotron2")
    fl = golden_flags(golden("t2_fwdmask_L100"))
    m = t2.Tacotron2(130, 0, r=1, attn_win=fl["attn_win"], attn_norm=fl["attn_norm"], forward_attn=fl["forward_attn"],
                     trans_agent=fl["trans_agent"], forward_attn_mask=fl["forward_attn_mask"],
                     location_attn=fl["location_attn"], max_batch=max_batch)
    return m.cuda().eval()


def test_persistent_griffin_lim_fresh_handles_ignore_freed_granules(audio_cfg):
    """Short-lived handles in sequence (the allocator hands a new handle the freed granule buffer of
    the last one, and every handle's tag salts start at 1): each persistent run, at 2 and at 3
    iterations, is bitwise the fused loop on the same input."""
    audio = load_pkg("audio")
    rng = np.random.Generator(np.random.PCG64(5))
    for k, iters in enumerate([2, 2, 3, 2, 3, 2]):
        mel = torch.from_numpy(rng.uniform(0, 1, size=(1, 100, 80)).astype(np.float32)).cuda()
        pu = rng.uniform(0, 1, size=(1, 1025, 100))
        ap = audio.AudioProcessor(**{**audio_cfg, "griffin_lim_iters": iters})
        a = ap.griffin_lim_batch(mel, [100], phase_u=pu)
        assert ap.last_gl_path() == "persistent"
        with _env(TTS_RESIDENT="0"):
            b = ap.griffin_lim_batch(mel, [100], phase_u=pu)
            assert ap.last_gl_path() == "fused"
        assert torch.equal(a, b), k
        del ap
        torch.cuda.synchronize()
