"""GPU parity of the Tacotron / TacotronGST path (SURVEY config 5; rows a17-a20) through the
C-ABI, against the reference's own outputs (tests/golden/gst_*.npz, taco_*.npz, made by
tests/golden/make_golden.py from the reference models) and the numpy oracle.

Tolerances as for Tacotron2 (north_star: alignments / stop tokens exact where they are decisions,
mel and linear spectrogram within 1e-4 relative RMS; held here to 4e-6, 10x the measured worst case):
step counts, per-step attention argmax and the stop decisions are compared exactly; alignments and stop
probabilities to max-abs 4e-6."""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden, golden_flags, load_pkg, rel_rms, weights_mod

pytestmark = pytest.mark.gpu

TACO_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "gst_*.npz")) +
                    glob.glob(os.path.join(GOLDEN, "taco_*.npz")))
RTOL = 4e-6  # 10x the worst measured (profiles/r05f_parity_report.jsonl: mel / linear <= 3e-7)
ATOL = 4e-6


def _model(fl, **kw):
    t = load_pkg("tacotron")
    cls = t.TacotronGST if fl["model"] == "TacotronGST" else t.Tacotron
    m = cls(130, fl["num_speakers"], r=fl["r"], memory_size=fl["memory_size"], attn_win=fl["attn_win"],
            attn_norm=fl["attn_norm"], forward_attn=fl["forward_attn"], trans_agent=fl["trans_agent"],
            forward_attn_mask=fl["forward_attn_mask"], location_attn=fl["location_attn"],
            prenet_type=fl.get("prenet_type", "original"), **kw)
    m.decoder.max_decoder_steps = fl["max_decoder_steps"]
    return m.cuda().eval()


def _inputs(z):
    sid = int(z["speaker_id"])
    style = torch.from_numpy(z["style_mel"])[None] if "style_mel" in z else None
    return (None if sid < 0 else torch.tensor([sid])), style


def _check_decoder(mel, align, stop, z, L):
    steps = z["align"].shape[0]
    assert align.shape[0] == steps, "step count differs from the reference"
    assert mel.shape[0] == z["mel"].shape[0]
    np.testing.assert_array_equal(align[:, :L].argmax(1), z["align"].argmax(1))
    assert np.abs(align[:, :L] - z["align"]).max() < ATOL
    np.testing.assert_array_equal(stop > 0.6, z["stop"] > 0.6)
    assert np.abs(stop - z["stop"]).max() < ATOL
    assert rel_rms(mel, z["mel"]) < RTOL


@pytest.mark.parametrize("case", TACO_CASES)
def test_full_inference_vs_reference(case):
    """TacotronGST.inference / Tacotron.inference(ids[, speaker, style_mel]) end to end."""
    z = golden(case)
    fl = golden_flags(z)
    m = _model(fl)
    sid, style = _inputs(z)
    x = torch.from_numpy(z["ids"])[None]
    if fl["model"] == "TacotronGST":
        mel, lin, align, stop = m.inference(x, speaker_ids=sid, style_mel=style)
    else:
        mel, lin, align, stop = m.inference(x, speaker_ids=sid)
    assert stop.shape == (1, z["align"].shape[0]) and lin.shape[2] == 1025
    _check_decoder(mel[0].cpu().numpy(), align[0].cpu().numpy(), stop[0].cpu().numpy(), z, len(z["ids"]))
    assert rel_rms(lin[0].cpu().numpy(), z["linear"]) < RTOL


@pytest.mark.parametrize("case", TACO_CASES)
def test_encoder_vs_reference(case):
    """Embedding + Prenet + CBHG (+ speaker embedding, + GST) vs the reference encoder outputs."""
    z = golden(case)
    fl = golden_flags(z)
    m = _model(fl)
    sid, style = _inputs(z)
    L = len(z["ids"])
    enc = m.encode(torch.from_numpy(z["ids"])[None].cuda(), [L], sid, style)
    assert rel_rms(enc[0].cpu().numpy(), z["enc"]) < RTOL


@pytest.mark.parametrize("case", TACO_CASES)
def test_decoder_and_postnet_vs_reference(case):
    """Decoder.inference from the reference's encoder outputs; PostCBHG from the reference's mel."""
    z = golden(case)
    m = _model(golden_flags(z))
    L = len(z["ids"])
    out = m.inference_batch(None, enc=torch.from_numpy(z["enc"])[None].cuda(), lens=[L], postnet=False)
    _check_decoder(out["mel"][0].cpu().numpy(), out["align"][0].cpu().numpy(), out["stop"][0].cpu().numpy(), z, L)
    mel = torch.from_numpy(z["mel"])[None].cuda()
    lin = m.postnet(mel, [mel.shape[1]])
    assert rel_rms(lin[0].cpu().numpy(), z["linear"]) < RTOL


def test_ragged_batch_matches_batch1():
    """A padded batch (decoder from the reference encoder outputs, then PostCBHG): every sentence
    gets its batch-1 reference result, whatever the others do (stop token at 1 step, alignment
    tail at 9 / 30 steps)."""
    cases = ["gst_L10_nostyle", "gst_L2_nostyle", "gst_L4_style", "gst_L10_nostyle"]
    zs = [golden(c) for c in cases]
    m = _model(golden_flags(zs[0]))
    lens = [len(z["ids"]) for z in zs]
    enc = torch.zeros(len(zs), max(lens), 256)
    for b, z in enumerate(zs):
        enc[b, :lens[b]] = torch.from_numpy(z["enc"])
    out = m.inference_batch(None, enc=enc.cuda(), lens=lens)
    assert out["steps"] == [z["align"].shape[0] for z in zs]
    for b, z in enumerate(zs):
        T = out["frames"][b]
        S = out["steps"][b]
        _check_decoder(out["mel"][b, :T].cpu().numpy(), out["align"][b, :S].cpu().numpy(),
                       out["stop"][b, :S].cpu().numpy(), z, lens[b])
        assert rel_rms(out["linear"][b, :T].cpu().numpy(), z["linear"]) < RTOL
        assert torch.all(out["linear"][b, T:] == 0)


def test_encoder_ragged_batch_with_style_and_speakers():
    """Encoder batch with per-sentence speakers and one style mel broadcast over the batch
    (models/tacotrongst.py:71-73, 86-88), each sentence at its own length, rows past it zero."""
    from oracle.tacotron_oracle import TacotronOracle
    w = weights_mod()
    fl = golden_flags(golden("gst_L24_style_spk"))
    m = _model(fl)
    o = TacotronOracle(w.tacotron_gst_weights(0, num_speakers=4), dtype=np.float32, **fl)
    lens = [17, 5, 31]
    ids = [w.synthetic_ids(L, 70 + L) for L in lens]
    style = w.synthetic_style_mel(47, 9)
    x = torch.zeros(3, 31, dtype=torch.long)
    for b, s in enumerate(ids):
        x[b, :lens[b]] = torch.from_numpy(s)
    enc = m.encode(x.cuda(), lens, [3, 0, 2], torch.from_numpy(style)[None]).cpu().numpy()
    for b, (L, spk) in enumerate(zip(lens, [3, 0, 2])):
        assert rel_rms(enc[b, :L], o.encoder(ids[b], spk, style)) < RTOL
        assert np.all(enc[b, L:] == 0)


def test_config5_batch32_vs_oracle():
    """SURVEY config 5 shape: B=32, L ~ U{60..160} (seed 4), speakers b mod 4, style mel
    [32, 200, 80] ~ U[0,1) (seed 4), the reference's 500-step cap.  Two sentences vs the oracle."""
    from oracle.tacotron_oracle import TacotronOracle
    w = weights_mod()
    gu = load_pkg("generic_utils")
    cfg = gu.default_config("config_tacotron_gst.json")
    m = gu.setup_model(130, 4, cfg).cuda().eval()
    lens = w.synthetic_lengths(32, 4)
    ids = [w.synthetic_ids(int(L), 200 + b) for b, L in enumerate(lens)]
    rng = np.random.Generator(np.random.PCG64(4))
    style = rng.uniform(0, 1, size=(32, 200, 80)).astype(np.float32)
    spk = [b % 4 for b in range(32)]
    out = m.inference_batch(ids, speaker_ids=spk, style_mel=torch.from_numpy(style))
    assert all(1 <= s <= 501 for s in out["steps"])
    assert torch.isfinite(out["linear"]).all()
    o = TacotronOracle(w.tacotron_gst_weights(0, num_speakers=4), dtype=np.float32, max_decoder_steps=500,
                       **{k: v for k, v in golden_flags(golden("gst_L24_style_spk")).items()
                          if k not in ("max_decoder_steps",)})
    for b in (0, 13):
        ref = o.inference(ids[b], spk[b], style[b])
        T = out["frames"][b]
        assert T == ref["mel"].shape[0]
        assert rel_rms(out["mel"][b, :T].cpu().numpy(), ref["mel"]) < RTOL
        assert rel_rms(out["linear"][b, :T].cpu().numpy(), ref["linear"]) < RTOL


def test_gst_synthesis_linear_griffin_lim(audio_cfg):
    """synthesis() on a TacotronGST: linear spectrogram -> inv_spectrogram (utils/synthesis.py:63-68)
    vs the oracle GL on the reference's linear output."""
    from oracle.griffin_lim_oracle import AudioOracle
    z = golden("gst_L4_style")
    fl = golden_flags(z)
    m = _model(fl)
    audio = load_pkg("audio")
    gu = load_pkg("generic_utils")
    C = gu.default_config("config_tacotron_gst.json")
    ap = audio.AudioProcessor(**{**C.audio, "griffin_lim_iters": 10})
    np.random.seed(5)
    wav, alignment, dec, post, stop = load_pkg("synthesis").synthesis(m, z["ids"], C, True, ap,
                                                                       style_wav=z["style_mel"])
    assert post.shape == z["linear"].shape and alignment.shape == z["align"].shape
    np.random.seed(5)
    ref = AudioOracle(**{**C.audio, "griffin_lim_iters": 10}).inv_spectrogram(z["linear"].T)
    assert rel_rms(wav, ref) < 1e-4


def test_melspectrogram_vs_reference_glue(audio_cfg):
    """HIP mel analysis (pre-emphasis FIR, float64 STFT, |D| complex64, mel, dB, normalise) vs the
    reference AudioProcessor.melspectrogram fixture."""
    z = golden("melspec")
    ap = load_pkg("audio").AudioProcessor(**audio_cfg)
    mel = ap.melspectrogram(z["wav"])
    assert mel.shape == z["mel"].shape
    assert np.abs(mel - z["mel"]).max() < 1e-5


def test_style_wav_synthesis_vs_oracle(tmp_path):
    """synthesis(..., style_wav=path) on a TacotronGST: wav file -> load_wav (+ trim) -> HIP mel
    analysis -> [1, 80, T] style mel read as rows of 80 values by the GST (gst_layers.py:60) ->
    encoder; the encoder output is checked against the oracle on the same wav."""
    import scipy.io.wavfile
    from oracle.griffin_lim_oracle import AudioOracle
    from oracle.tacotron_oracle import TacotronOracle
    gu = load_pkg("generic_utils")
    C = gu.default_config("config_tacotron_gst.json")
    rng = np.random.Generator(np.random.PCG64(12))
    n = 22050
    t = np.arange(n) / 22050.0
    y = (0.4 * np.sin(2 * np.pi * 330 * t) * (t > 0.2) * (t < 0.8) + 0.001 * rng.standard_normal(n))
    path = str(tmp_path / "style.wav")
    scipy.io.wavfile.write(path, 22050, (y * 32767).astype(np.int16))
    ap = load_pkg("audio").AudioProcessor(**C.audio)
    x = ap.load_wav(path)
    assert 0 < len(x) < n  # trimmed (do_trim_silence is on in config_tacotron_gst.json)
    style = load_pkg("synthesis").compute_style_mel(path, ap)
    assert style.shape == (1, 80, 1 + len(x) // 275)
    ref_mel = AudioOracle(**C.audio).melspectrogram(x)
    assert np.abs(style[0].cpu().numpy() - ref_mel).max() < 1e-5
    fl = golden_flags(golden("gst_L10_nostyle"))
    m = _model(fl)
    ids = weights_mod().synthetic_ids(14, 3)
    enc = m.encode(torch.from_numpy(ids)[None].cuda(), [14], None, style)
    o = TacotronOracle(weights_mod().tacotron_gst_weights(0), dtype=np.float32, **fl)
    ref = o.encoder(ids, None, ref_mel.astype(np.float32).reshape(-1, 80))
    assert rel_rms(enc[0].cpu().numpy(), ref) < RTOL


def test_fused_query_matches_separate_query_launch(monkeypatch):
    """The TacotronGST step computes query_layer(h_att) inside the attention launch (transposed
    weight, 8 k-slices summed in a fixed order); TTS_GST_FUSED_QUERY=0 keeps the separate GEMM
    launch.  Both on a B=8 config-5-shaped batch (speakers, style mel): identical step counts and
    stop decisions, spectrograms within 1e-5 relative RMS (fp32 summation order only)."""
    w = weights_mod()
    gu = load_pkg("generic_utils")
    cfg = gu.default_config("config_tacotron_gst.json")
    lens = w.synthetic_lengths(8, 4)
    ids = [w.synthetic_ids(int(L), 300 + b) for b, L in enumerate(lens)]
    style = torch.from_numpy(np.random.Generator(np.random.PCG64(8)).uniform(0, 1, size=(8, 200, 80)).astype(np.float32))
    spk = [b % 4 for b in range(8)]
    outs = []
    for fused in ("1", "0"):
        monkeypatch.setenv("TTS_GST_FUSED_QUERY", fused)
        m = gu.setup_model(130, 4, cfg).cuda().eval()
        m.decoder.max_decoder_steps = 120
        outs.append(m.inference_batch(ids, speaker_ids=spk, style_mel=style))
    a, b = outs
    assert a["steps"] == b["steps"] and a["frames"] == b["frames"]
    for b_ in range(8):
        T = a["frames"][b_]
        assert rel_rms(a["linear"][b_, :T].cpu().numpy(), b["linear"][b_, :T].cpu().numpy()) < 1e-5
        assert rel_rms(a["mel"][b_, :T].cpu().numpy(), b["mel"][b_, :T].cpu().numpy()) < 1e-5


def _config5_batch(n, seed=4):
    w = weights_mod()
    lens = w.synthetic_lengths(n, seed)
    ids = [w.synthetic_ids(int(L), 200 + b) for b, L in enumerate(lens)]
    rng = np.random.Generator(np.random.PCG64(seed))
    style = torch.from_numpy(rng.uniform(0, 1, size=(n, 200, 80)).astype(np.float32))
    return ids, [b % 4 for b in range(n)], style


def _decode_enc(m, enc, lens):
    out = m.inference_batch(None, enc=enc, lens=lens, postnet=False)
    return out, dict(m.last_timing)


@pytest.mark.parametrize("B", [32, 5])
def test_resident_decoder_matches_multilaunch(monkeypatch, B):
    """The resident decoder (tacotron_resident.hip: one launch, each XCD decoding up to 4 sentences
    with the step weights on its 32 CUs) against the per-step multi-launch path on the same encoder
    outputs (config-5 shaped batch, full 500-step cap): identical step counts, stop decisions and
    alignment argmax per step; mel, stop and alignment within 1e-5 (the two differ only in fp32
    summation order and in alpha = w / sum(w) without the sigmoid normaliser, which cancels)."""
    gu = load_pkg("generic_utils")
    cfg = gu.default_config("config_tacotron_gst.json")
    ids, spk, style = _config5_batch(B)
    m = gu.setup_model(130, 4, cfg).cuda().eval()
    L = max(len(x) for x in ids)
    x = torch.zeros(B, L, dtype=torch.long)
    lens = [len(s) for s in ids]
    for b, s in enumerate(ids):
        x[b, :lens[b]] = torch.from_numpy(s)
    enc = m.encode(x.cuda(), lens, spk, style)
    res, tr = _decode_enc(m, enc, lens)
    assert tr["resident"], "resident decoder did not run"
    monkeypatch.setenv("TTS_RESIDENT", "0")
    m2 = gu.setup_model(130, 4, cfg).cuda().eval()
    ml, tm = _decode_enc(m2, enc, lens)
    assert not tm["resident"]
    assert res["steps"] == ml["steps"]
    for b in range(B):
        T, S = res["frames"][b], res["steps"][b]
        a1 = res["align"][b, :S, :lens[b]].cpu().numpy()
        a2 = ml["align"][b, :S, :lens[b]].cpu().numpy()
        np.testing.assert_array_equal(a1.argmax(1), a2.argmax(1))
        assert np.abs(a1 - a2).max() < 1e-5
        assert torch.all(res["align"][b, :S, lens[b]:] == 0)
        s1, s2 = res["stop"][b, :S].cpu().numpy(), ml["stop"][b, :S].cpu().numpy()
        np.testing.assert_array_equal(s1 > 0.6, s2 > 0.6)
        assert np.abs(s1 - s2).max() < 1e-5
        assert rel_rms(res["mel"][b, :T].cpu().numpy(), ml["mel"][b, :T].cpu().numpy()) < 1e-5
        assert torch.all(res["mel"][b, T:] == 0)


def test_resident_decoder_deterministic_and_timeout_rerun(monkeypatch):
    """Two resident runs of the same batch are bitwise identical (fixed reduction orders); with a
    1-tick hand-off timeout every wait fails, the kernel drains with its status and the batch re-runs
    on the multi-launch path, bitwise equal to a TTS_RESIDENT=0 handle."""
    gu = load_pkg("generic_utils")
    cfg = gu.default_config("config_tacotron_gst.json")
    ids, spk, style = _config5_batch(6, seed=9)
    m = gu.setup_model(130, 4, cfg).cuda().eval()
    m.decoder.max_decoder_steps = 150
    L = max(len(x) for x in ids)
    x = torch.zeros(6, L, dtype=torch.long)
    lens = [len(s) for s in ids]
    for b, s in enumerate(ids):
        x[b, :lens[b]] = torch.from_numpy(s)
    enc = m.encode(x.cuda(), lens, spk, style)
    r1, t1 = _decode_enc(m, enc, lens)
    r2, t2 = _decode_enc(m, enc, lens)
    assert t1["resident"] and t2["resident"]
    for k in ("mel", "stop", "align"):
        assert torch.equal(r1[k], r2[k]), k
    monkeypatch.setenv("TTS_DEC_WAIT_TICKS", "1")
    mt = gu.setup_model(130, 4, cfg).cuda().eval()
    mt.decoder.max_decoder_steps = 150
    rt, tt = _decode_enc(mt, enc, lens)
    assert not tt["resident"]
    monkeypatch.delenv("TTS_DEC_WAIT_TICKS")
    monkeypatch.setenv("TTS_RESIDENT", "0")
    m0 = gu.setup_model(130, 4, cfg).cuda().eval()
    m0.decoder.max_decoder_steps = 150
    r0, _ = _decode_enc(m0, enc, lens)
    assert rt["steps"] == r0["steps"]
    for k in ("mel", "stop", "align"):
        assert torch.equal(rt[k], r0[k]), k
