"""GPU: the resident single-launch batch-1 decoder (csrc/resident_decoder.hip) against the
multi-launch path (TTS_RESIDENT=0 at create) and the oracle.

Both implementations compute the same fp32 step in different reduction orders, so frame counts,
attention argmax paths and stop decisions must be identical and mel / alignments agree to fp32
rounding; the oracle tolerance is the parity suite's (mel relative RMS 4e-6)."""
import os

import numpy as np
import pytest
import torch

from conftest import golden, golden_flags, load_pkg, rel_rms, weights_mod
from oracle.tacotron2_oracle import Tacotron2Oracle

pytestmark = pytest.mark.gpu

FL = None


def _flags():
    global FL
    if FL is None:
        FL = golden_flags(golden("t2_fwdmask_L100"))  # synthesis configuration (synthesize.py:86)
    return FL


def _model(resident):
    t2 = load_pkg("tacotron2")
    fl = _flags()
    old = os.environ.get("TTS_RESIDENT")
    os.environ["TTS_RESIDENT"] = "1" if resident else "0"
    try:
        m = t2.Tacotron2(130, 0, r=1, attn_win=fl["attn_win"], attn_norm=fl["attn_norm"],
                         forward_attn=fl["forward_attn"], trans_agent=fl["trans_agent"],
                         forward_attn_mask=fl["forward_attn_mask"], location_attn=fl["location_attn"])
        m.decoder.max_decoder_steps = fl["max_decoder_steps"]
        m = m.cuda().eval()
        m.inference_batch([[5, 6]])  # creates the native handles while the variable is set
    finally:
        if old is None:
            del os.environ["TTS_RESIDENT"]
        else:
            os.environ["TTS_RESIDENT"] = old
    return m


@pytest.fixture(scope="module")
def models():
    return _model(True), _model(False)


@pytest.mark.parametrize("L", [2, 3, 5, 12, 64, 100, 129, 200, 256])
def test_resident_matches_multilaunch(models, L):
    res, ml = models
    w = weights_mod()
    ids = w.synthetic_ids(L, 300 + L)
    a = res.inference_batch([ids])
    assert res.last_timing["resident"], "the resident decoder did not serve a batch-1 call"
    b = ml.inference_batch([ids])
    assert not ml.last_timing["resident"]
    assert a["frames"] == b["frames"]
    T = a["frames"][0]
    np.testing.assert_array_equal(a["align"][0, :T, :L].cpu().numpy().argmax(1),
                                  b["align"][0, :T, :L].cpu().numpy().argmax(1))
    np.testing.assert_array_equal(a["stop"][0, :T].cpu().numpy() > 0.5, b["stop"][0, :T].cpu().numpy() > 0.5)
    assert np.abs(a["align"][0, :T].cpu().numpy() - b["align"][0, :T].cpu().numpy()).max() < 1e-5
    assert rel_rms(a["mel"][0, :T].cpu().numpy(), b["mel"][0, :T].cpu().numpy()) < 1e-5
    assert rel_rms(a["mel_post"][0, :T].cpu().numpy(), b["mel_post"][0, :T].cpu().numpy()) < 1e-5


@pytest.mark.parametrize("L", [150, 256])
def test_resident_vs_oracle_long(models, L):
    """Positions >= 128 take the energy loop's global-memory branch; L = 256 is the maximum."""
    res, _ = models
    w = weights_mod()
    ids = w.synthetic_ids(L, 900 + L)
    out = res.inference_batch([ids])
    assert res.last_timing["resident"]
    ref = Tacotron2Oracle(w.tacotron2_weights(0), dtype=np.float32, **_flags()).inference(ids)
    T = out["frames"][0]
    assert T == ref["mel"].shape[0]
    np.testing.assert_array_equal(out["align"][0, :T, :L].cpu().numpy().argmax(1), ref["align"].argmax(1))
    assert rel_rms(out["mel"][0, :T].cpu().numpy(), ref["mel"]) < 4e-6
    assert rel_rms(out["mel_post"][0, :T].cpu().numpy(), ref["mel_post"]) < 4e-6


def test_resident_deterministic_and_batches_unaffected(models):
    res, ml = models
    w = weights_mod()
    ids = w.synthetic_ids(100, 1)
    x = res.inference_batch([ids])
    y = res.inference_batch([ids])
    assert torch.equal(x["mel"], y["mel"]) and torch.equal(x["align"], y["align"])
    # a batch of 2 on the same handle takes the resident batch decoder (resident_batch.hip, round 6)
    # and matches the multi-launch one; its encoder is the batched resident BiLSTM (XCD-parallel,
    # MFMA gate rows) where `ml` runs the per-step launches, so the two agree to fp32
    # reduction-order noise rather than bit for bit
    ids2 = w.synthetic_ids(40, 2)
    z = res.inference_batch([ids, ids2])
    assert res.last_timing["resident_kind"] == 2
    zz = ml.inference_batch([ids, ids2])
    assert list(z["frames"]) == list(zz["frames"])
    for b, T in enumerate(z["frames"]):
        a, r = z["mel"][b, :int(T)].double(), zz["mel"][b, :int(T)].double()
        d = float((a - r).norm() / r.norm())
        assert d < 1e-5, (b, d)  # the encoder's reduction order only
    # ... and both against the oracle: exact frame counts and attention argmax, mel at 4e-6
    for b, x_ids in enumerate((ids, ids2)):
        ref = Tacotron2Oracle(w.tacotron2_weights(0), dtype=np.float32, **_flags()).inference(x_ids)
        T, L = int(z["frames"][b]), len(x_ids)
        assert T == ref["mel"].shape[0]
        for out in (z, zz):
            np.testing.assert_array_equal(out["align"][b, :T, :L].cpu().numpy().argmax(1), ref["align"].argmax(1))
            assert rel_rms(out["mel"][b, :T].cpu().numpy(), ref["mel"]) < 4e-6
    assert torch.equal(res.inference_batch([ids, ids2])["mel"], z["mel"])  # deterministic
    # and a batch-1 call afterwards is resident again and unchanged
    x2 = res.inference_batch([ids])
    assert res.last_timing["resident"] and torch.equal(x2["mel"], x["mel"])
