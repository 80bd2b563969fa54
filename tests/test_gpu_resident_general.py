"""GPU: the resident decoder's general attention form (resident.h, round 5) — every Tacotron2
attention configuration other than synthesize.py's masked one, at batch 1, in one persistent launch
with the attention spread over each XCD's 32 CUs.

Against the reference's own outputs (tests/golden/t2_*.npz, made by tests/golden/make_golden.py
from /root/reference): frame counts, per-step attention argmax and stop decisions exact; mel,
mel_post, alignments and stop probabilities at the parity suite's tolerances.  Against the
multi-launch path of the same configuration (TTS_RESIDENT_GEN=0 at create): same integers, floats
within fp32 reduction-order noise.  The Synthesizer.tts() configuration (config_tacotron2.json as
is: forward attention, sigmoid, mask OFF; server/synthesizer.py:46-66) and the constructor default
(location-sensitive + softmax, models/tacotron2.py:17,23) are pinned at L=100 on their full
reference runs (1000 / 300 steps)."""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden, golden_flags, load_pkg, rel_rms

pytestmark = pytest.mark.gpu

MEL_RTOL = 4e-6  # 10x the worst measured over every fixture and path (profiles/r05f_parity_report.jsonl)
ALIGN_ATOL = 4e-6
SAME_RTOL = 1e-5  # resident vs multi-launch: the same fp32 step, different reduction orders
SAME_ATOL = 1e-5


def _general(case):
    fl = golden_flags(golden(case))
    return not (fl["forward_attn"] and fl["forward_attn_mask"] and fl["attn_norm"] == "sigmoid"
                and not fl["location_attn"] and not fl["attn_win"] and not fl["trans_agent"])


GEN_CASES = [c for c in sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "t2_*.npz")))
             if _general(c)]


def _model(fl, gen=True):
    t2 = load_pkg("tacotron2")
    old = os.environ.get("TTS_RESIDENT_GEN")
    os.environ["TTS_RESIDENT_GEN"] = "1" if gen else "0"
    try:
        m = t2.Tacotron2(130, 0, r=1, attn_win=fl["attn_win"], attn_norm=fl["attn_norm"],
                         forward_attn=fl["forward_attn"], trans_agent=fl["trans_agent"],
                         forward_attn_mask=fl["forward_attn_mask"], location_attn=fl["location_attn"])
        m.decoder.max_decoder_steps = fl["max_decoder_steps"]
        m.max_len = 256
        m = m.cuda().eval()
        m.inference_batch([[5, 6]])  # creates the native handles while the variable is set
    finally:
        if old is None:
            del os.environ["TTS_RESIDENT_GEN"]
        else:
            os.environ["TTS_RESIDENT_GEN"] = old
    return m


def _run(m, z):
    enc = torch.from_numpy(z["enc"]).cuda()[None]
    out = m.inference_batch(None, enc=enc, lens=[len(z["ids"])])
    return out


def _check_vs_reference(out, z):
    T = out["frames"][0]
    assert T == z["mel"].shape[0], "frame count differs from the reference"
    L = len(z["ids"])
    al = out["align"][0, :T, :L].cpu().numpy()
    np.testing.assert_array_equal(al.argmax(1), z["align"].argmax(1))
    assert np.abs(al - z["align"]).max() < ALIGN_ATOL
    st = out["stop"][0, :T].cpu().numpy()
    np.testing.assert_array_equal(st > 0.5, z["stop"] > 0.5)
    assert np.abs(st - z["stop"]).max() < ALIGN_ATOL
    assert rel_rms(out["mel"][0, :T].cpu().numpy(), z["mel"]) < MEL_RTOL
    assert rel_rms(out["mel_post"][0, :T].cpu().numpy(), z["mel_post"]) < MEL_RTOL


@pytest.mark.parametrize("case", GEN_CASES)
def test_general_resident_vs_reference(case):
    z = golden(case)
    m = _model(golden_flags(z))
    out = _run(m, z)
    assert m.last_timing["resident"], "the general resident form did not serve this batch-1 call"
    _check_vs_reference(out, z)


@pytest.mark.parametrize("case", GEN_CASES)
def test_general_resident_vs_multilaunch(case):
    z = golden(case)
    fl = golden_flags(z)
    res, ml = _model(fl, True), _model(fl, False)
    a = _run(res, z)
    assert res.last_timing["resident"]
    b = _run(ml, z)
    assert not ml.last_timing["resident"]
    assert a["frames"] == b["frames"]
    T, L = a["frames"][0], len(z["ids"])
    aa, ab = a["align"][0, :T, :L].cpu().numpy(), b["align"][0, :T, :L].cpu().numpy()
    np.testing.assert_array_equal(aa.argmax(1), ab.argmax(1))
    assert np.abs(aa - ab).max() < SAME_ATOL
    sa, sb = a["stop"][0, :T].cpu().numpy(), b["stop"][0, :T].cpu().numpy()
    np.testing.assert_array_equal(sa > 0.5, sb > 0.5)
    assert np.abs(sa - sb).max() < SAME_ATOL
    for k in ("mel", "mel_post"):
        assert rel_rms(a[k][0, :T].cpu().numpy(), b[k][0, :T].cpu().numpy()) < SAME_RTOL, k


def test_general_resident_deterministic():
    z = golden("t2_nomask_L100")
    m = _model(golden_flags(z))
    a = _run(m, z)
    b = _run(m, z)
    T = a["frames"][0]
    for k in ("mel", "mel_post", "align", "stop"):
        assert torch.equal(a[k][0, :T], b[k][0, :T]), k


@pytest.mark.parametrize("L", [2, 3, 31, 32, 33, 64, 129, 255, 256])
def test_general_resident_lengths_vs_multilaunch(L):
    """Position ownership edges: L below / at / above one position per CU (32), full waves, the
    256 maximum; location + forward attention + transition agent (every general state at once)."""
    fl = golden_flags(golden("t2_loc_fwd_ta_L100"))
    fl = dict(fl, max_decoder_steps=2 * L + 40)
    w = load_pkg("weights")
    ids = w.synthetic_ids(L, 700 + L)
    res, ml = _model(fl, True), _model(fl, False)
    a = res.inference_batch([ids])
    assert res.last_timing["resident"]
    b = ml.inference_batch([ids])
    assert a["frames"] == b["frames"]
    T = a["frames"][0]
    np.testing.assert_array_equal(a["align"][0, :T, :L].argmax(-1).cpu().numpy(),
                                  b["align"][0, :T, :L].argmax(-1).cpu().numpy())
    assert (a["align"][0, :T, :L] - b["align"][0, :T, :L]).abs().max().item() < SAME_ATOL
    assert rel_rms(a["mel_post"][0, :T].cpu().numpy(), b["mel_post"][0, :T].cpu().numpy()) < SAME_RTOL


def test_synthesizer_configuration_is_resident(tmp_path):
    """Synthesizer(config) (server/synthesizer.py:30-66, config_tacotron2.json: forward attention,
    sigmoid, mask off, 3000-step cap): a one-sentence request decodes on the resident decoder."""
    synth = load_pkg("synthesis")
    gu = load_pkg("generic_utils")
    from test_cli import _write_model_files
    cfg_path, ckpt, _ = _write_model_files(tmp_path)
    conf = tmp_path / "conf.json"
    conf.write_text('{"tts_path": "%s", "tts_file": "%s", "tts_config": "config.json", "wavernn_lib_path": "",'
                    ' "use_cuda": true, "port": 5002}' % (tmp_path, ckpt.name))
    s = synth.Synthesizer(gu.load_config(str(conf)))
    assert s.tts_model.flags["forward_attn_mask"] is False and s.tts_model.decoder.max_decoder_steps == 3000
    wav = s.tts("It took me quite a long time to develop a voice and now that I have it I am not silent.")
    assert len(wav.getvalue()) > 44
    assert s.tts_model.last_timing["resident"], "Synthesizer.tts() did not decode on the resident path"


def test_general_resident_past_2048_steps():
    """Runs past 2048 steps (the Synthesizer's 3000-step cap, mask off): the hand-off tags wrap the
    step count; two consecutive launches (odd and even tag salts) match the multi-launch path."""
    fl = dict(golden_flags(golden("t2_nomask_L100")), max_decoder_steps=2100)
    w = load_pkg("weights")
    ids = w.synthetic_ids(60, 4242)
    res, ml = _model(fl, True), _model(fl, False)
    b = ml.inference_batch([ids])
    for _ in range(2):
        a = res.inference_batch([ids])
        assert res.last_timing["resident"]
        assert a["frames"] == b["frames"] == [2100]
        T = a["frames"][0]
        np.testing.assert_array_equal(a["align"][0, :T, :60].argmax(-1).cpu().numpy(),
                                      b["align"][0, :T, :60].argmax(-1).cpu().numpy())
        assert rel_rms(a["mel_post"][0, :T].cpu().numpy(), b["mel_post"][0, :T].cpu().numpy()) < SAME_RTOL
