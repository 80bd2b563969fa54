"""CPU: pin the oracle against the reference's own outputs (tests/golden, made by
tests/golden/make_golden.py from /root/reference).  Runs anywhere, no GPU."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden, golden_flags, rel_rms, tacotron2_config, weights_mod
from oracle.griffin_lim_oracle import AudioOracle, mel_filters, stft, istft
from oracle.tacotron2_oracle import Tacotron2Oracle

T2_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "t2_*.npz")))
# the 3000-step fixture (Synthesizer.tts()'s cap) pins the GPU path directly; the CPU restatements
# take ~2 min on it (checked when it was made): TTS_SLOW_ORACLE=1 includes it here
T2_CASES = [c for c in T2_CASES if not c.endswith("_cap3000") or os.environ.get("TTS_SLOW_ORACLE") == "1"]


@pytest.mark.parametrize("case", T2_CASES)
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_tacotron2_oracle_matches_reference(case, dtype):
    z = golden(case)
    fl = golden_flags(z)
    sd = weights_mod().tacotron2_weights(0, location_attn=fl["location_attn"], trans_agent=fl["trans_agent"])
    o = Tacotron2Oracle(sd, dtype=dtype, **fl)
    enc = o.encoder(z["ids"])
    assert rel_rms(enc, z["enc"]) < 1e-6
    mel, stop, align = o.decoder(z["enc"])
    # integer/index outputs: exact
    assert mel.shape == z["mel"].shape, "frame count differs from the reference"
    np.testing.assert_array_equal(align.argmax(1), z["align"].argmax(1))
    np.testing.assert_array_equal(stop > 0.5, z["stop"] > 0.5)
    # float outputs: fp32 reference vs restatement
    assert rel_rms(mel, z["mel"]) < 1e-5
    assert np.abs(align - z["align"]).max() < 1e-5
    assert np.abs(stop - z["stop"]).max() < 1e-5
    assert rel_rms(o.postnet(z["mel"]), z["mel_post"]) < 1e-5


def test_stop_rule_frame_count_2L_plus_22():
    """With the forward-attention mask (synthesize.py:86) the reference stops at 2L+22."""
    for case in ("t2_fwdmask_L12", "t2_fwdmask_L40", "t2_fwdmask_L100"):
        z = golden(case)
        assert z["mel"].shape[0] == 2 * len(z["ids"]) + 22


def test_forward_mask_wraparound_step0():
    """Step-0 alignment is nonzero exactly at [0,1,2,3,L-1] (common_layers.py:207-213 wrap)."""
    z = golden("t2_fwdmask_L40")
    nz = np.nonzero(z["align"][0])[0].tolist()
    assert nz == [0, 1, 2, 3, 39]


@pytest.mark.parametrize("case", sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "gl_*mel*.npz"))))
def test_gl_oracle_matches_reference_glue(case, audio_cfg):
    z = golden(case)
    ap = AudioOracle(**{**audio_cfg, "griffin_lim_iters": int(z["iters"])})
    np.random.seed(int(z["phase_seed"]))
    pu = np.random.rand(1025, z["mel"].shape[1])
    wav = ap.inv_mel_spectrogram(z["mel"], pu)
    assert wav.dtype == np.float64 and wav.shape == z["wav"].shape
    assert rel_rms(wav, z["wav"]) < 1e-12
    if "S" in z:
        assert rel_rms(ap.mel_magnitude(z["mel"]), z["S"]) < 1e-6


def test_gl_linear_path(audio_cfg):
    z = golden("gl_linear_it3")
    ap = AudioOracle(**{**audio_cfg, "griffin_lim_iters": 3})
    np.random.seed(int(z["phase_seed"]))
    pu = np.random.rand(*z["spec"].shape)
    assert rel_rms(ap.inv_spectrogram(z["spec"], pu), z["wav"]) < 1e-12


def test_inverse_preemphasis_and_save_wav(audio_cfg):
    ap = AudioOracle(**audio_cfg)
    z = golden("preemph")
    np.testing.assert_array_equal(ap.inv_preemphasis(z["x"]), z["y"])
    z = golden("save_wav")
    np.testing.assert_array_equal(AudioOracle.wav_to_int16(z["wav"]), z["pcm"])


def test_librosa_restatement_properties(audio_cfg):
    """Unpinned against librosa; check the published invariants instead."""
    M = mel_filters(22050, 2048, 80, 0.0, 8000.0)
    assert M.shape == (80, 1025) and (M >= 0).all()
    # Slaney area norm: each filter integrates (over Hz) to ~1 -> sum * bin width ~ 1
    bw = 22050 / 2048
    assert np.allclose(M.sum(1) * bw, 1.0, atol=0.15)
    # stft -> istft round trip reconstructs the signal (COLA with the sum-square normalisation)
    rng = np.random.Generator(np.random.PCG64(0))
    y = rng.standard_normal(275 * 40).astype(np.float32)
    D = stft(y, 2048, 275, 1102)
    assert D.dtype == np.complex64 and D.shape == (1025, 41)
    y2 = istft(D, 275, 1102)
    assert y2.shape == y.shape and rel_rms(y2, y) < 1e-5


TACO_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "gst_*.npz")) +
                    glob.glob(os.path.join(GOLDEN, "taco_*.npz")))


def taco_oracle(z, dtype=np.float64):
    from oracle.tacotron_oracle import TacotronOracle
    fl = dict(golden_flags(z))
    bn = fl.pop("prenet_type", "original") == "bn"
    sd = weights_mod().tacotron_gst_weights(0, num_speakers=fl["num_speakers"], r=fl["r"],
                                            memory_size=fl["memory_size"], location_attn=fl["location_attn"],
                                            trans_agent=fl["trans_agent"], gst=fl["model"] == "TacotronGST",
                                            prenet_bn=bn)
    return TacotronOracle(sd, dtype=dtype, **fl)


@pytest.mark.parametrize("case", TACO_CASES)
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_tacotron_gst_oracle_matches_reference(case, dtype):
    """Tacotron / TacotronGST restatement vs the reference (models/tacotron*.py) on its own fixtures."""
    z = golden(case)
    o = taco_oracle(z, dtype)
    sid = int(z["speaker_id"])
    enc = o.encoder(z["ids"], None if sid < 0 else sid, z["style_mel"] if "style_mel" in z else None)
    assert rel_rms(enc, z["enc"]) < 1e-5
    if "gst" in z:
        assert rel_rms(o.gst(z["style_mel"]), z["gst"]) < 1e-5
    mel, stop, align = o.decoder(z["enc"])
    assert mel.shape == z["mel"].shape, "frame count differs from the reference"
    np.testing.assert_array_equal(align.argmax(1), z["align"].argmax(1))
    assert rel_rms(mel, z["mel"]) < 1e-5
    assert np.abs(align - z["align"]).max() < 1e-5
    assert np.abs(stop - z["stop"]).max() < 1e-5
    assert rel_rms(o.postnet(z["mel"]), z["linear"]) < 1e-5


def test_tacotron_stop_rule_variants():
    """The fixtures cover each exit of layers/tacotron.py:464-469: stop token (L=2, one step),
    alignment tail (L=4/10) and the max_decoder_steps cap (+1 step)."""
    assert golden("gst_L2_nostyle")["align"].shape[0] == 1
    z = golden("gst_L4_style")
    assert z["align"][-1, -1] > 0.6 and z["align"].shape[0] < 41
    z = golden("gst_L24_style_spk")
    assert z["align"].shape[0] == golden_flags(z)["max_decoder_steps"] + 1


def test_tacotron2_truncated_oracle_matches_reference():
    """Continuous mode (Tacotron2.inference_truncated over three texts): encoder BiLSTM state and
    decoder states carry over (models/tacotron2.py:75-89)."""
    z = golden("trunc_t2_3texts")
    fl = golden_flags(z)
    o = Tacotron2Oracle(weights_mod().tacotron2_weights(0), dtype=np.float32, **fl)
    res = o.inference_truncated([z[f"ids{i}"] for i in range(3)])
    for i, r in enumerate(res):
        assert r["mel"].shape == z[f"mel{i}"].shape
        np.testing.assert_array_equal(r["align"].argmax(1), z[f"align{i}"].argmax(1))
        assert rel_rms(r["mel"], z[f"mel{i}"]) < 1e-5
        assert rel_rms(r["mel_post"], z[f"mel_post{i}"]) < 1e-5
    # the carry matters: text 1 alone differs from text 1 after text 0
    alone = o.inference(z["ids1"])
    assert rel_rms(alone["mel"], z["mel1"]) > 1e-3


def test_melspectrogram_oracle_matches_reference_glue(audio_cfg):
    """AudioProcessor.melspectrogram (utils/audio.py:146-152; compute_style_mel's analysis) vs the
    reference run with the librosa restatement (glue pinned, librosa internals unpinned)."""
    z = golden("melspec")
    ap = AudioOracle(**audio_cfg)
    mel = ap.melspectrogram(z["wav"])
    assert mel.shape == z["mel"].shape == (80, 1 + len(z["wav"]) // 275)
    assert np.abs(mel - z["mel"]).max() < 1e-12


@pytest.mark.parametrize("case", ["tf_fwdmask_L12", "tf_loc_softmax_L20", "tf_win_fwdmask_L16"])
def test_teacher_forced_oracle_matches_reference(case):
    """Decoder.forward (teacher forcing, layers/tacotron2.py:227-247) restated vs the reference run on
    the same encoder output and teacher mel (tests/golden/tf_*.npz)."""
    z = golden(case)
    fl = golden_flags(z)
    o = Tacotron2Oracle(weights_mod().tacotron2_weights(0, location_attn=fl["location_attn"]), dtype=np.float64,
                        **fl)
    mel, stop, align = o.decoder(z["enc"], teacher=z["teacher"])
    assert mel.shape == z["mel"].T.shape and stop.shape == z["stop"].shape and align.shape == z["align"].shape
    assert np.abs(mel - z["mel"].T).max() < 1e-5
    assert np.abs(stop - z["stop"]).max() < 1e-5
    assert np.abs(align - z["align"]).max() < 1e-6
    np.testing.assert_array_equal(align.argmax(1), z["align"].argmax(1))
    assert np.abs(o.postnet(mel) - z["mel_post"].T).max() < 1e-5


BN_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "t2bn_*.npz")))


@pytest.mark.parametrize("case", BN_CASES)
def test_tacotron2_oracle_prenet_bn_matches_reference(case):
    """prenet_type "bn" (LinearBN layers, common_layers.py:28-52, 66-70; eval BatchNorm1d): both
    oracles against the reference run (tests/golden/make_golden.py prenet_bn)."""
    from oracle.tacotron2_torch import Tacotron2TorchCPU
    z = golden(case)
    fl = golden_flags(z)
    sd = weights_mod().tacotron2_weights(0, prenet_bn=True)
    assert "decoder.prenet.layers.1.bn.running_var" in sd
    for res in (Tacotron2Oracle(sd, dtype=np.float32, **fl).inference(z["ids"]),
                Tacotron2TorchCPU(sd, **fl).inference(z["ids"])):
        assert res["mel"].shape == z["mel"].shape
        np.testing.assert_array_equal(res["align"].argmax(1), z["align"].argmax(1))
        assert rel_rms(res["mel"], z["mel"]) < 1e-4
        assert rel_rms(res["mel_post"], z["mel_post"]) < 1e-4
    # the BatchNorm matters: the same weights without it give another utterance
    plain = {k: v for k, v in sd.items() if ".bn." not in k}
    res = Tacotron2Oracle(plain, dtype=np.float32, **fl).inference(z["ids"])
    assert res["mel"].shape != z["mel"].shape or rel_rms(res["mel"], z["mel"]) > 1e-2


SPK_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "t2spk_*.npz")))


@pytest.mark.parametrize("case", SPK_CASES)
def test_tacotron2_oracle_speakers_match_reference(case):
    """Tacotron2 with speaker embeddings (models/tacotron2.py:32-34, 91-100): the oracles against the
    reference run with 4 speakers (tests/golden/make_golden.py speakers)."""
    from oracle.tacotron2_torch import Tacotron2TorchCPU
    z = golden(case)
    fl = golden_flags(z)
    sd = weights_mod().tacotron2_weights(0, num_speakers=4)
    spk = int(z["speaker_id"])
    o = Tacotron2Oracle(sd, dtype=np.float32, **fl)
    assert rel_rms(o.encoder(z["ids"], spk), z["enc"]) < 1e-6
    for res in (o.inference(z["ids"], spk), Tacotron2TorchCPU(sd, **fl).inference(z["ids"], spk)):
        assert res["mel"].shape == z["mel"].shape
        np.testing.assert_array_equal(res["align"].argmax(1), z["align"].argmax(1))
        assert rel_rms(res["mel"], z["mel"]) < 1e-4
        assert rel_rms(res["mel_post"], z["mel_post"]) < 1e-4


def test_prenet_bn_fold_algebra():
    """The create-time fold of an eval-mode BatchNorm1d into the preceding linear layer (decoder_api.hip /
    tacotron_api.hip: fold_linear_bn): W' = diag(s) W, b' = s (b - mean) + beta, s = gamma / sqrt(var + eps),
    equals Linear -> BatchNorm1d (common_layers.py:28-52) on random inputs, with and without a linear bias."""
    rng = np.random.Generator(np.random.PCG64(11))
    W = rng.standard_normal((256, 80)).astype(np.float64)
    g, be = rng.uniform(0.8, 1.2, 256), rng.uniform(-0.1, 0.1, 256)
    mu, var = rng.uniform(-0.1, 0.1, 256), rng.uniform(0.5, 1.5, 256)
    x = rng.standard_normal((7, 80))
    for b in (None, rng.uniform(-0.1, 0.1, 256)):
        y = x @ W.T + (0 if b is None else b)
        ref = (y - mu) / np.sqrt(var + 1e-5) * g + be
        s = g / np.sqrt(var + 1e-5)
        Wf = W * s[:, None]
        bf = s * ((0 if b is None else b) - mu) + be
        np.testing.assert_allclose(x @ Wf.T + bf, ref, rtol=1e-12, atol=1e-12)
