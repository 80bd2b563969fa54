"""GPU parity: the HIP path (through the C-ABI) against the reference's golden outputs and the
oracle.  Tolerances (north_star: "alignments/stop-tokens bit-exact, mel and waveform within
1e-4 RMS"): integer/index outputs — frame count, per-step attention argmax, stop decisions — are
compared exactly; float outputs of a different fp32 reduction order cannot be bitwise equal, so
alignments/stop tokens are held to max-abs 4e-6 and mel to relative RMS 4e-6 (10x the measured
worst case, profiles/r05f_parity_report.jsonl), the waveform to north_star's relative RMS 1e-4
(absolute RMS is vacuous here: the random-weight waveform has RMS ~1e-5)."""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden, golden_flags, load_pkg, rel_rms, weights_mod
from oracle.griffin_lim_oracle import AudioOracle
from oracle.tacotron2_oracle import Tacotron2Oracle

pytestmark = pytest.mark.gpu

T2_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "t2_*.npz")))
# model half: about 10x the worst error measured over every reference fixture on every path
# (profiles/r05f_parity_report.jsonl: mel / mel_post relative RMS <= 3.4e-7, alignments <= 4.2e-7,
# stop probabilities <= 6e-8 max-abs); the waveform keeps north_star's 1e-4 (Griffin-Lim amplifies
# the fp32 rounding of its input about 100x over 60 iterations)
MEL_RTOL = 4e-6
ALIGN_ATOL = 4e-6
WAV_RTOL = 1e-4


def _model(fl, **kw):
    t2 = load_pkg("tacotron2")
    m = t2.Tacotron2(130, 0, r=1, attn_win=fl["attn_win"], attn_norm=fl["attn_norm"],
                     forward_attn=fl["forward_attn"], trans_agent=fl["trans_agent"],
                     forward_attn_mask=fl["forward_attn_mask"], location_attn=fl["location_attn"], **kw)
    m.decoder.max_decoder_steps = fl["max_decoder_steps"]
    return m.cuda().eval()


def _check_decoder(out, b, z):
    T = out["frames"][b]
    assert T == z["mel"].shape[0], "frame count differs from the reference"
    L = len(z["ids"])
    al = out["align"][b, :T, :L].cpu().numpy()
    np.testing.assert_array_equal(al.argmax(1), z["align"].argmax(1))
    assert np.abs(al - z["align"]).max() < ALIGN_ATOL
    st = out["stop"][b, :T].cpu().numpy()
    np.testing.assert_array_equal(st > 0.5, z["stop"] > 0.5)
    assert np.abs(st - z["stop"]).max() < ALIGN_ATOL
    assert rel_rms(out["mel"][b, :T].cpu().numpy(), z["mel"]) < MEL_RTOL
    assert rel_rms(out["mel_post"][b, :T].cpu().numpy(), z["mel_post"]) < MEL_RTOL


@pytest.mark.parametrize("case", T2_CASES)
def test_decoder_postnet_vs_reference(case):
    """Decoder.inference + Postnet from the reference's own encoder outputs."""
    z = golden(case)
    m = _model(golden_flags(z))
    enc = torch.from_numpy(z["enc"]).cuda()[None]
    out = m.inference_batch(None, enc=enc, lens=[len(z["ids"])])
    _check_decoder(out, 0, z)


@pytest.mark.parametrize("case", ["t2_fwdmask_L12", "t2_fwdmask_L100", "t2_loc_fwd_ta_L24"])
def test_full_inference_vs_reference(case):
    """Tacotron2.inference(ids) end to end (encoder on the GPU, decoder + postnet in HIP)."""
    z = golden(case)
    m = _model(golden_flags(z))
    mel, mel_post, align, stop = m.inference(torch.from_numpy(z["ids"])[None])
    assert mel.shape == (1,) + z["mel"].shape and stop.shape == (1, z["mel"].shape[0], 1)
    assert rel_rms(mel[0].cpu().numpy(), z["mel"]) < MEL_RTOL
    assert rel_rms(mel_post[0].cpu().numpy(), z["mel_post"]) < MEL_RTOL
    np.testing.assert_array_equal(align[0].cpu().numpy().argmax(1), z["align"].argmax(1))


@pytest.mark.parametrize("case", ["t2_fwdmask_L12", "t2_fwdmask_L40", "t2_fwdmask_L100"])
def test_encoder_vs_reference(case):
    """HIP encoder (embedding + 3 conv/BN/ReLU + BiLSTM) vs the reference's encoder outputs."""
    z = golden(case)
    m = _model(golden_flags(z))
    L = len(z["ids"])
    enc = m.encode(torch.from_numpy(z["ids"])[None].cuda(), [L])
    assert rel_rms(enc[0].cpu().numpy(), z["enc"]) < MEL_RTOL


def test_encoder_ragged_batch():
    """Padded batch: each sentence encoded at its own length (reverse LSTM starts at L_b-1),
    rows past L_b are zero."""
    cases = ["t2_fwdmask_L40", "t2_fwdmask_L100", "t2_fwdmask_L12"]
    zs = [golden(c) for c in cases]
    m = _model(golden_flags(zs[0]))
    lens = [len(z["ids"]) for z in zs]
    ids = torch.zeros(len(zs), max(lens), dtype=torch.long)
    for b, z in enumerate(zs):
        ids[b, :lens[b]] = torch.from_numpy(z["ids"])
    enc = m.encode(ids.cuda(), lens).cpu().numpy()
    for b, z in enumerate(zs):
        assert rel_rms(enc[b, :lens[b]], z["enc"]) < MEL_RTOL
        assert np.all(enc[b, lens[b]:] == 0)


def test_batched_ragged_decoder_matches_batch1():
    """A padded batch: every sentence gets exactly its batch-1 reference result."""
    cases = ["t2_fwdmask_L40", "t2_fwdmask_L12", "t2_fwdmask_L100", "t2_fwdmask_L12", "t2_fwdmask_L40"]
    zs = [golden(c) for c in cases]
    m = _model(golden_flags(zs[0]))
    Lmax = max(len(z["ids"]) for z in zs)
    enc = torch.zeros(len(zs), Lmax, 512)
    for b, z in enumerate(zs):
        enc[b, :len(z["ids"])] = torch.from_numpy(z["enc"])
    out = m.inference_batch(None, enc=enc.cuda(), lens=[len(z["ids"]) for z in zs])
    for b, z in enumerate(zs):
        _check_decoder(out, b, z)


def test_batch64_lengths_property():
    """Config-3 shape (B=64, L ~ U{60..160}): every sentence stops at 2L+22, oracle on two."""
    w = weights_mod()
    lens = w.synthetic_lengths(64, 2)
    ids = [w.synthetic_ids(int(L), 100 + b) for b, L in enumerate(lens)]
    fl = golden_flags(golden("t2_fwdmask_L100"))
    m = _model(fl)
    out = m.inference_batch(ids)
    assert out["frames"] == [2 * int(L) + 22 for L in lens]
    assert torch.isfinite(out["mel_post"]).all()
    o = Tacotron2Oracle(w.tacotron2_weights(0), dtype=np.float32, **fl)
    for b in (0, 37):
        ref = o.inference(ids[b])
        T = out["frames"][b]
        assert T == ref["mel"].shape[0]
        assert rel_rms(out["mel"][b, :T].cpu().numpy(), ref["mel"]) < MEL_RTOL
        assert rel_rms(out["mel_post"][b, :T].cpu().numpy(), ref["mel_post"]) < MEL_RTOL


@pytest.mark.parametrize("L", [2, 3, 4, 5])
def test_shortest_sentences_vs_oracle(L):
    """L=2..5: the forward mask's negative-index wrap ((n-2) % L) and the clipped window [n-1, n+2]
    overlap at these lengths; the context must still only sum the surviving positions."""
    w = weights_mod()
    fl = golden_flags(golden("t2_fwdmask_L12"))
    m = _model(fl)
    ids = w.synthetic_ids(L, 50 + L)
    out = m.inference_batch([ids])
    ref = Tacotron2Oracle(w.tacotron2_weights(0), dtype=np.float32, **fl).inference(ids)
    T = out["frames"][0]
    assert T == ref["mel"].shape[0]
    np.testing.assert_array_equal(out["align"][0, :T, :L].cpu().numpy().argmax(1), ref["align"].argmax(1))
    assert rel_rms(out["mel"][0, :T].cpu().numpy(), ref["mel"]) < MEL_RTOL
    assert rel_rms(out["mel_post"][0, :T].cpu().numpy(), ref["mel_post"]) < MEL_RTOL


def test_sharded_synthesis_single_rank(audio_cfg):
    """sharding.synthesize_sharded over a 1-rank RCCL group equals the single-process batch."""
    import torch.distributed as dist
    sh = load_pkg("sharding")
    synth = load_pkg("synthesis")
    audio = load_pkg("audio")
    w = weights_mod()
    fl = golden_flags(golden("t2_fwdmask_L12"))
    m = _model(fl)
    ap = audio.AudioProcessor(**{**audio_cfg, "griffin_lim_iters": 5})
    ids = [w.synthetic_ids(L, 7 + L) for L in (9, 17, 4)]
    store = dist.TCPStore("127.0.0.1", 0, 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1)
    try:
        pcm, info = sh.synthesize_sharded(m, ap, ids, seed=11)
    finally:
        dist.destroy_process_group()
    wavs, _ = synth.synthesize_batch(m, ap, ids, seed=11, phase="device")
    np.testing.assert_array_equal(pcm, sh.join_int16(wavs))
    assert info["partition"] == [[0, 1, 2]]


@pytest.mark.parametrize("case", sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "gl_*mel*.npz"))))
def test_griffin_lim_vs_reference_glue(case, audio_cfg):
    """inv_mel_spectrogram with the reference's np.random phases (seeded) vs the reference's
    AudioProcessor run on the librosa restatement."""
    z = golden(case)
    audio = load_pkg("audio")
    ap = audio.AudioProcessor(**{**audio_cfg, "griffin_lim_iters": int(z["iters"])})
    np.random.seed(int(z["phase_seed"]))
    wav = ap.inv_mel_spectrogram(z["mel"])
    assert wav.dtype == np.float64 and wav.shape == z["wav"].shape
    assert rel_rms(wav, z["wav"]) < WAV_RTOL
    pcm = load_pkg("synthesis").wav_to_int16(wav)
    ref_pcm = AudioOracle.wav_to_int16(z["wav"])
    assert np.abs(pcm.astype(np.int32) - ref_pcm).max() <= 2


def test_griffin_lim_linear_path(audio_cfg):
    z = golden("gl_linear_it3")
    audio = load_pkg("audio")
    ap = audio.AudioProcessor(**{**audio_cfg, "griffin_lim_iters": 3})
    np.random.seed(int(z["phase_seed"]))
    assert rel_rms(ap.inv_spectrogram(z["spec"]), z["wav"]) < WAV_RTOL


def test_griffin_lim_batched_ragged_60_iters(audio_cfg):
    """Ragged batch at the metric's 60 iterations vs the oracle one sentence at a time."""
    audio = load_pkg("audio")
    ap = audio.AudioProcessor(**audio_cfg)  # griffin_lim_iters = 60
    o = AudioOracle(**audio_cfg)
    rng = np.random.Generator(np.random.PCG64(7))
    Fs = [46, 13, 80, 2, 31]
    Fmax = max(Fs)
    mel = np.zeros((len(Fs), Fmax, 80), np.float32)
    pu = np.zeros((len(Fs), 1025, Fmax))
    for b, F in enumerate(Fs):
        mel[b, :F] = rng.uniform(0, 1, size=(F, 80))
        pu[b, :, :F] = rng.uniform(0, 1, size=(1025, F))
    wav = ap.griffin_lim_batch(torch.from_numpy(mel).cuda(), Fs, phase_u=pu).cpu().numpy()
    for b, F in enumerate(Fs):
        ref = o.inv_mel_spectrogram(mel[b, :F].T, pu[b, :, :F])
        n = ap.hop_length * (F - 1)
        assert rel_rms(wav[b, :n], ref) < WAV_RTOL, (b, F)
        assert np.all(wav[b, n:] == 0)


def device_phases(seed, F, nb=1025):
    """numpy restatement of griffin_lim.hip hash_uniform (sentence 0): U[k, f] of the device phases."""
    idx = (np.arange(nb, dtype=np.uint64)[:, None] * np.uint64(1048576) + np.arange(F, dtype=np.uint64)[None, :])
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15) * (idx + np.uint64(1))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def test_griffin_lim_configs1_persistent_vs_oracle(audio_cfg):
    """the exact configs[1] Griffin-Lim — the reference's own mel_post of the L=100
    sentence (T = 222 frames), 60 iterations, on the persistent loop — against the oracle's
    inv_mel_spectrogram with the same phases."""
    z = golden("t2_fwdmask_L100")
    mel = z["mel_post"].astype(np.float32)
    F = mel.shape[0]
    assert F == 222
    ap = load_pkg("audio").AudioProcessor(**audio_cfg)  # 60 iterations
    pu = np.random.Generator(np.random.PCG64(11)).uniform(0, 1, size=(1, 1025, F))
    wav = ap.griffin_lim_batch(torch.from_numpy(mel[None]).cuda(), [F], phase_u=pu).cpu().numpy()[0]
    assert ap.last_gl_path() == "persistent"
    ref = AudioOracle(**audio_cfg).inv_mel_spectrogram(mel.T, pu[0])
    assert rel_rms(wav, ref) < WAV_RTOL


@pytest.mark.parametrize("Fs", [[300], [512], [190, 140]])
def test_griffin_lim_persistent_two_per_cu_vs_oracle(audio_cfg, monkeypatch, Fs):
    """257..512 frames in all: the persistent loop's two-workgroups-per-CU form
    (gl_persistent2_kernel), against the oracle per sentence and bitwise against the fused
    per-iteration loop (TTS_RESIDENT=0)."""
    audio = load_pkg("audio")
    ap = audio.AudioProcessor(**{**audio_cfg, "griffin_lim_iters": 20})
    rng = np.random.Generator(np.random.PCG64(sum(Fs)))
    Fmax = max(Fs)
    mel = np.zeros((len(Fs), Fmax, 80), np.float32)
    pu = np.zeros((len(Fs), 1025, Fmax))
    for b, F in enumerate(Fs):
        mel[b, :F] = rng.uniform(0, 1, size=(F, 80))
        pu[b, :, :F] = rng.uniform(0, 1, size=(1025, F))
    wav = ap.griffin_lim_batch(torch.from_numpy(mel).cuda(), Fs, phase_u=pu).cpu()
    assert ap.last_gl_path() == "persistent"
    monkeypatch.setenv("TTS_RESIDENT", "0")
    fused = ap.griffin_lim_batch(torch.from_numpy(mel).cuda(), Fs, phase_u=pu).cpu()
    assert ap.last_gl_path() != "persistent"
    assert torch.equal(wav, fused)
    o = AudioOracle(**{**audio_cfg, "griffin_lim_iters": 20})
    for b, F in enumerate(Fs):
        n = ap.hop_length * (F - 1)
        assert rel_rms(wav[b, :n].numpy(), o.inv_mel_spectrogram(mel[b, :F].T, pu[b, :, :F])) < WAV_RTOL, b


def test_synthesize_native_configs1_vs_oracle(audio_cfg):
    """configs[1] end to end on the benched path (tts_synth_run: resident decoder, postnet and the
    persistent Griffin-Lim enqueued behind it, device phases) against the oracle chain: the
    reference's mel_post through inv_mel_spectrogram with the device's phases (hash restated)."""
    z = golden("t2_fwdmask_L100")
    m = _model(golden_flags(z))
    ap = load_pkg("audio").AudioProcessor(**audio_cfg)
    wav, frames = m.synthesize_native([z["ids"]], ap, seed=21)
    F = z["mel"].shape[0]
    assert frames == [F]
    ref = AudioOracle(**audio_cfg).inv_mel_spectrogram(z["mel_post"].T, device_phases(21, F))
    assert rel_rms(wav.cpu().numpy()[0], ref) < WAV_RTOL


def test_end_to_end_synthesis_vs_oracle(audio_cfg):
    """ids -> wav through the whole HIP path vs the oracle chain (L=12, 60 GL iterations).

    Mean over four numpy phase draws: with the model half within 3.1e-7 of the reference, the
    single-draw waveform distance is a heavy-tailed realization of Griffin-Lim's sensitivity
    (3e-6 .. 1e-4 across draws for the same mel, profiles/r05_e2e_wave_probe.txt)."""
    z = golden("t2_fwdmask_L12")
    fl = golden_flags(z)
    m = _model(fl)
    audio = load_pkg("audio")
    ap = audio.AudioProcessor(**audio_cfg)
    errs = []
    for seed in (3, 4, 5, 6):
        np.random.seed(seed)
        wavs, info = load_pkg("synthesis").synthesize_batch(m, ap, [z["ids"]], phase="numpy")
        np.random.seed(seed)
        ref = AudioOracle(**audio_cfg).inv_mel_spectrogram(z["mel_post"].T)
        assert info["frames"] == [z["mel"].shape[0]]
        errs.append(rel_rms(wavs[0], ref))
    assert float(np.mean(errs)) < WAV_RTOL, errs


def test_native_errors_are_raised():
    t2 = load_pkg("tacotron2")
    m = t2.Tacotron2(130, 0, r=1, attn_norm="sigmoid", forward_attn=True, forward_attn_mask=True,
                     location_attn=False).cuda()
    with pytest.raises(ValueError):
        m.inference_batch([[5]])  # L=1 has no alpha[n-2] in the reference
    bad = m.state_dict()
    bad["decoder.attention_rnn.weight_ih"] = torch.zeros(4096, 700)
    with pytest.raises(RuntimeError):
        m.load_state_dict(bad)


def test_inference_truncated_vs_reference():
    """Tacotron2.inference_truncated over three consecutive texts (continuous mode) vs the
    reference: encoder BiLSTM state, decoder LSTM states, context and memory carry over."""
    z = golden("trunc_t2_3texts")
    m = _model(golden_flags(z))
    for i in range(3):
        mel, mel_post, align, stop = m.inference_truncated(torch.from_numpy(z[f"ids{i}"])[None])
        assert mel.shape[1] == z[f"mel{i}"].shape[0]
        np.testing.assert_array_equal(align[0].cpu().numpy().argmax(1), z[f"align{i}"].argmax(1))
        assert rel_rms(mel[0].cpu().numpy(), z[f"mel{i}"]) < MEL_RTOL
        assert rel_rms(mel_post[0].cpu().numpy(), z[f"mel_post{i}"]) < MEL_RTOL
    # a fresh inference() afterwards is unaffected
    z0 = golden("t2_fwdmask_L12")
    mel, mel_post, _, _ = m.inference(torch.from_numpy(z0["ids"])[None])
    assert rel_rms(mel_post[0].cpu().numpy(), z0["mel_post"]) < MEL_RTOL


@pytest.mark.parametrize("coef", [0.97, 0.98, 0.995])
@pytest.mark.parametrize("F", [17, 100, 300])
def test_deemphasis_scan_chunks(audio_cfg, coef, F):
    """The chunk-parallel de-emphasis (griffin_lim.hip: preemph_scan_kernel) vs scipy's sequential
    lfilter on the same float32 signal: the signal comes from a run with pre-emphasis off (same
    phases), so the only difference is the recurrence.  0.995 needs more look-back than a tile and
    takes the one-chunk-per-sentence scan; 17 frames fit one chunk, 100 and 300 span several."""
    from scipy.signal import lfilter
    audio = load_pkg("audio")
    rng = np.random.Generator(np.random.PCG64(F))
    mel = torch.from_numpy(rng.uniform(0, 1, size=(1, F, 80)).astype(np.float32)).cuda()
    pu = rng.uniform(0, 1, size=(1, 1025, F))
    base = audio.AudioProcessor(**{**audio_cfg, "griffin_lim_iters": 2, "preemphasis": 0.0})
    emph = audio.AudioProcessor(**{**audio_cfg, "griffin_lim_iters": 2, "preemphasis": coef})
    y = base.griffin_lim_batch(mel, [F], phase_u=pu).cpu().numpy()[0]
    wav = emph.griffin_lim_batch(mel, [F], phase_u=pu).cpu().numpy()[0]
    n = base.hop_length * (F - 1)
    ref = lfilter([1.0], [1.0, -coef], y[:n])
    err = np.abs(wav[:n] - ref)
    bad = np.nonzero(err > 1e-12 * np.max(np.abs(ref)))[0]
    assert bad.size == 0, (bad.size, bad[:4], bad[-4:], err.max())
    assert np.all(wav[n:] == 0)


@pytest.mark.parametrize("cases", [["t2_fwdmask_L100"], ["t2_fwdmask_L40", "t2_fwdmask_L12", "t2_fwdmask_L100"]])
def test_synthesize_native_matches_staged(audio_cfg, cases):
    """tts_synth_run (ids -> wav in one call) is bitwise the staged path: inference_batch, then
    griffin_lim_batch with the same device-phase seed (batch 1 = resident decoder + persistent GL;
    a ragged batch 3 = multi-launch decoder + compacted GL input)."""
    zs = [golden(c) for c in cases]
    m = _model(golden_flags(zs[0]))
    audio = load_pkg("audio")
    ap = audio.AudioProcessor(**{**audio_cfg, "griffin_lim_iters": 10})
    ids = [z["ids"] for z in zs]
    wav, frames = m.synthesize_native(ids, ap, seed=5)
    out = m.inference_batch(ids)
    ref = ap.griffin_lim_batch(out["mel_post"], out["frames"], seed=5)
    assert frames == out["frames"] == [z["mel"].shape[0] for z in zs]
    assert wav.shape == ref.shape
    assert torch.equal(wav, ref)


def test_synthesize_native_server_cap(audio_cfg):
    """at the server's max_decoder_steps=3000 (Synthesizer, server/synthesizer.py) the
    batch-1 postnet enqueued behind the decoder is sized by the small-kernel bound, not by the
    3021-frame cap; waveforms (222 frames: persistent Griffin-Lim in the hook; 322 frames:
    redone after the wait) are bitwise inference_batch + griffin_lim_batch."""
    fl = dict(golden_flags(golden("t2_fwdmask_L100")), max_decoder_steps=3000)
    m = _model(fl)
    ap = load_pkg("audio").AudioProcessor(**{**audio_cfg, "griffin_lim_iters": 6})
    for k, ids in enumerate((golden("t2_fwdmask_L100")["ids"], weights_mod().synthetic_ids(150, 7))):
        wav, frames = m.synthesize_native([ids], ap, seed=30 + k)
        out = m.inference_batch([ids])
        ref = ap.griffin_lim_batch(out["mel_post"], out["frames"], seed=30 + k)
        assert frames == out["frames"]
        assert torch.equal(wav, ref), k


def test_synthesize_native_back_to_back(audio_cfg):
    """tts_synth_run returns once Griffin-Lim is enqueued (the next call's host work and encoder
    overlap it; its stages run on the synth handle's stream): back-to-back calls with alternating
    batch shapes, each output taken on the caller's stream right after its call, each bitwise the
    staged path; then a staged call on the same handles right after a pipelined one."""
    zs = {c: golden(c) for c in ("t2_fwdmask_L100", "t2_fwdmask_L40", "t2_fwdmask_L12")}
    m = _model(golden_flags(zs["t2_fwdmask_L100"]))
    audio = load_pkg("audio")
    ap = audio.AudioProcessor(**{**audio_cfg, "griffin_lim_iters": 6})
    seq = [["t2_fwdmask_L100"], ["t2_fwdmask_L40", "t2_fwdmask_L12"], ["t2_fwdmask_L100"], ["t2_fwdmask_L12"]]
    outs = []
    for k, cases in enumerate(seq):
        wav, frames = m.synthesize_native([zs[c]["ids"] for c in cases], ap, seed=20 + k)
        outs.append((wav.clone(), frames))  # ordered after the call on the caller's stream
    m.synthesize_native([zs["t2_fwdmask_L40"]["ids"]], ap, seed=99)
    for k, cases in enumerate(seq):
        ids = [zs[c]["ids"] for c in cases]
        out = m.inference_batch(ids)
        ref = ap.griffin_lim_batch(out["mel_post"], out["frames"], seed=20 + k)
        wav, frames = outs[k]
        assert frames == out["frames"]
        assert torch.equal(wav, ref), k


def test_synthesize_native_pipelined_cross_stream(audio_cfg):
    """sync=False back to back across the cross-stream path: jobs above 512 frames run Griffin-Lim on
    the synth handle's second stream while the next call's encoder / decoder / postnet run (batch-1
    ones on the resident decoder), the stage buffers alternate by call parity; small jobs in between
    take the same-stream persistent Griffin-Lim.  Every waveform, cloned on the caller's stream right
    after its call, is bitwise inference_batch + griffin_lim_batch at the same seed."""
    w = weights_mod()
    z = {c: golden(c)["ids"] for c in ("t2_fwdmask_L100", "t2_fwdmask_L12", "t2_fwdmask_L40")}
    z["L150"] = w.synthetic_ids(260, 7)  # 2L + 22 frames under the mask: above 512
    z["L140"] = w.synthetic_ids(140, 8)  # 302 frames: the same-stream persistent loop, two per CU
    m = _model(golden_flags(golden("t2_fwdmask_L100")))
    audio = load_pkg("audio")
    ap = audio.AudioProcessor(**{**audio_cfg, "griffin_lim_iters": 6})
    seq = [["L150"], ["L140"], ["t2_fwdmask_L100"] * 3, ["t2_fwdmask_L12"], ["L150", "t2_fwdmask_L40"],
           ["L140"], ["t2_fwdmask_L12"]]
    outs = []
    for k, cases in enumerate(seq):
        wav, frames = m.synthesize_native([z[c] for c in cases], ap, seed=50 + k, sync=False)
        outs.append((wav.clone(), frames))
    m.synth_sync()
    assert sum(outs[0][1]) > 512 and sum(outs[2][1]) > 512 and 256 < sum(outs[1][1]) <= 512 and sum(outs[3][1]) <= 256
    for k, cases in enumerate(seq):
        ids = [z[c] for c in cases]
        out = m.inference_batch(ids)
        ref = ap.griffin_lim_batch(out["mel_post"], out["frames"], seed=50 + k)
        wav, frames = outs[k]
        assert frames == out["frames"], k
        assert torch.equal(wav, ref), k


@pytest.mark.parametrize("cap", [30, 31, 33, 40, 60])
def test_synthesize_native_stop_near_cap(audio_cfg, cap):
    """The stop rule fires within 20 steps of max_decoder_steps (the `elif` cap of
    layers/tacotron2.py:271-277 is skipped once every stop flag is set, so the decoder may run up to
    max_steps + 20 steps): tts_synth_run's waveform buffer holds those frames, the frame count is the
    oracle's at the same cap, and the waveform is bitwise the staged path."""
    z = golden("t2_nomask_L12")
    fl = dict(golden_flags(z), max_decoder_steps=cap)
    m = _model(fl)
    ap = load_pkg("audio").AudioProcessor(**{**audio_cfg, "griffin_lim_iters": 4})
    o = Tacotron2Oracle(weights_mod().tacotron2_weights(0), dtype=np.float32, **fl)
    T = o.inference(z["ids"])["mel"].shape[0]
    wav, frames = m.synthesize_native([z["ids"]], ap, seed=3)
    assert frames == [T]
    out = m.inference_batch([z["ids"]])
    ref = ap.griffin_lim_batch(out["mel_post"], out["frames"], seed=3)
    assert out["frames"] == [T] and torch.equal(wav, ref)
    # every flag is set from step 30 on: a cap of 30 ends the loop there, any later cap lets the
    # stop count run to 51 frames (31 + 20: the widest overshoot at cap 31)
    assert T == (30 if cap == 30 else 51)


TF_CASES = ["tf_fwdmask_L12", "tf_loc_softmax_L20", "tf_win_fwdmask_L16"]


@pytest.mark.parametrize("case", TF_CASES)
def test_decoder_forward_teacher_forcing_vs_reference(case):
    """Decoder.forward (teacher forcing, layers/tacotron2.py:227-247) vs the reference run on the same
    encoder output and teacher mel: mel [B, 80, T], stop LOGITS [B, T], alignments [B, T, L]."""
    z = golden(case)
    fl = golden_flags(z)
    m = _model(fl)
    mel, stop, align = m.decoder_forward(torch.from_numpy(z["enc"])[None], torch.from_numpy(z["teacher"])[None])
    assert tuple(mel.shape) == (1,) + z["mel"].shape and tuple(stop.shape) == (1,) + z["stop"].shape
    assert tuple(align.shape) == (1,) + z["align"].shape
    assert rel_rms(mel[0].cpu().numpy(), z["mel"]) < MEL_RTOL
    np.testing.assert_array_equal(align[0].cpu().numpy().argmax(1), z["align"].argmax(1))
    assert np.abs(align[0].cpu().numpy() - z["align"]).max() < ALIGN_ATOL
    assert np.abs(stop[0].cpu().numpy() - z["stop"]).max() < ALIGN_ATOL * max(1.0, np.abs(z["stop"]).max())


def test_tacotron2_forward_ragged_batch_teacher_forcing():
    """Tacotron2.forward (models/tacotron2.py:47-60, eval) on a padded batch: the fixture sentence
    (its first 20 teacher frames: teacher forcing is causal, so its outputs are the fixture's first 20
    steps) next to a shorter sentence checked against the oracle's forward at its own length."""
    z = golden("tf_fwdmask_L12")
    fl = golden_flags(z)
    m = _model(fl)
    w = weights_mod()
    ids2 = w.synthetic_ids(7, 88)
    T = 20
    teacher2 = np.random.Generator(np.random.PCG64(89)).uniform(0, 1, size=(T, 80)).astype(np.float32)
    text = torch.zeros(2, 12, dtype=torch.long)
    text[0] = torch.from_numpy(z["ids"])
    text[1, :7] = torch.from_numpy(ids2)
    mels = torch.from_numpy(np.stack([z["teacher"][:T], teacher2]))
    mel, mel_post, align, stop = m.forward(text, torch.tensor([12, 7]), mels)
    assert tuple(mel.shape) == (2, T, 80) and tuple(align.shape) == (2, T, 12) and tuple(stop.shape) == (2, T)
    assert rel_rms(mel[0].cpu().numpy(), z["mel"].T[:T]) < MEL_RTOL
    np.testing.assert_array_equal(align[0].cpu().numpy().argmax(1), z["align"][:T].argmax(1))
    ref = Tacotron2Oracle(w.tacotron2_weights(0), dtype=np.float32, **fl).forward(ids2, teacher2)
    assert rel_rms(mel[1].cpu().numpy(), ref["mel"]) < MEL_RTOL
    assert rel_rms(mel_post[1].cpu().numpy(), ref["mel_post"]) < MEL_RTOL
    al = align[1, :, :7].cpu().numpy()
    np.testing.assert_array_equal(al.argmax(1), ref["align"].argmax(1))
    assert np.abs(stop[1].cpu().numpy() - ref["stop"]).max() < 1e-3


@pytest.mark.gpu
def test_tacotron2_forward_batch20_teacher_forcing_mirrors():
    """Above 16 sentences the decoder GEMMs read fragment-order mirrors of their inputs
    (csrc/sgemm.h: Seg::pf), kept beside the row-major state by every producer; under teacher
    forcing the prenet runs on the teacher frame at every step and must keep the pre1 mirror in
    step.  The fixture sentence and a shorter one inside a ragged batch of 20, against the
    reference fixture and the oracle's forward (models/tacotron2.py:47-60)."""
    z = golden("tf_fwdmask_L12")
    fl = golden_flags(z)
    m = _model(fl)
    w = weights_mod()
    T, B = 20, 20
    rng = np.random.Generator(np.random.PCG64(90))
    text = torch.zeros(B, 12, dtype=torch.long)
    mels = np.zeros((B, T, 80), np.float32)
    lens = []
    ids2 = w.synthetic_ids(7, 88)
    teacher2 = np.random.Generator(np.random.PCG64(89)).uniform(0, 1, size=(T, 80)).astype(np.float32)
    for b in range(B):
        if b == 0:
            ids, mels[b] = z["ids"], z["teacher"][:T]
        elif b == 1:
            ids, mels[b] = ids2, teacher2
        else:
            ids = w.synthetic_ids(int(rng.integers(2, 13)), 100 + b)
            mels[b] = rng.uniform(0, 1, size=(T, 80)).astype(np.float32)
        text[b, :len(ids)] = torch.from_numpy(ids)
        lens.append(len(ids))
    mel, mel_post, align, stop = m.forward(text, torch.tensor(lens), torch.from_numpy(mels))
    assert tuple(mel.shape) == (B, T, 80)
    assert rel_rms(mel[0].cpu().numpy(), z["mel"].T[:T]) < MEL_RTOL
    np.testing.assert_array_equal(align[0].cpu().numpy().argmax(1), z["align"][:T].argmax(1))
    ref = Tacotron2Oracle(w.tacotron2_weights(0), dtype=np.float32, **fl).forward(ids2, teacher2)
    assert rel_rms(mel[1].cpu().numpy(), ref["mel"]) < MEL_RTOL
    assert rel_rms(mel_post[1].cpu().numpy(), ref["mel_post"]) < MEL_RTOL
    np.testing.assert_array_equal(align[1, :, :7].cpu().numpy().argmax(1), ref["align"].argmax(1))
    assert np.abs(stop[1].cpu().numpy() - ref["stop"]).max() < 1e-3


def test_batched_varlen_convs_bitwise(monkeypatch):
    """configs[2]-shaped batch (B=64, L ~ U{60..160}): the encoder and postnet convs on varlen 64-frame
    tiles (conv1d.hip: conv_vl_kernel) give bitwise the padded-tile kernel's results."""
    w = weights_mod()
    lens = w.synthetic_lengths(64, 2)
    ids = [w.synthetic_ids(int(L), 100 + b) for b, L in enumerate(lens)]
    fl = golden_flags(golden("t2_fwdmask_L100"))
    m = _model(fl, max_batch=64)
    a = m.inference_batch(ids)
    monkeypatch.setenv("TTS_CONV_VL", "0")
    b = m.inference_batch(ids)
    assert a["frames"] == b["frames"]
    assert torch.equal(a["mel_post"], b["mel_post"]) and torch.equal(a["mel"], b["mel"])


def _speaker_model():
    t2 = load_pkg("tacotron2")
    fl = golden_flags(golden("t2spk_fwdmask_L24_s2"))
    m = t2.Tacotron2(130, 4, r=1, attn_win=fl["attn_win"], attn_norm=fl["attn_norm"], forward_attn=fl["forward_attn"],
                     trans_agent=fl["trans_agent"], forward_attn_mask=fl["forward_attn_mask"],
                     location_attn=fl["location_attn"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in weights_mod().tacotron2_weights(0, num_speakers=4).items()})
    return m.cuda().eval()


def test_speaker_embedding_batch_vs_reference():
    """Tacotron2 with 4 speakers: a ragged batch of two sentences with different speakers through
    inference_batch (native tts_encoder_add_speakers) against the reference's own outputs."""
    zs = [golden("t2spk_fwdmask_L24_s2"), golden("t2spk_fwdmask_L40_s0")]
    m = _speaker_model()
    out = m.inference_batch([z["ids"] for z in zs], speaker_ids=[int(z["speaker_id"]) for z in zs])
    for b, z in enumerate(zs):
        T = out["frames"][b]
        assert T == z["mel"].shape[0]
        np.testing.assert_array_equal(out["align"][b, :T, :len(z["ids"])].cpu().numpy().argmax(1), z["align"].argmax(1))
        assert rel_rms(out["mel"][b, :T].cpu().numpy(), z["mel"]) < MEL_RTOL
        assert rel_rms(out["mel_post"][b, :T].cpu().numpy(), z["mel_post"]) < MEL_RTOL


def test_speaker_embedding_synthesize_native_vs_oracle(audio_cfg):
    """The one-call synthesis with a speaker (tts_synth_run_speakers, batch 1: resident path) against
    the oracle chain on the reference's mel_post with the device's phases."""
    z = golden("t2spk_fwdmask_L24_s2")
    m = _speaker_model()
    ap = load_pkg("audio").AudioProcessor(**audio_cfg)
    wav, frames = m.synthesize_native([z["ids"]], ap, seed=5, speaker_ids=[int(z["speaker_id"])])
    wav = wav.clone()  # (the returned waveform is a view of the model's buffer)
    F = z["mel"].shape[0]
    assert frames == [F]
    ref = AudioOracle(**audio_cfg).inv_mel_spectrogram(z["mel_post"].T, device_phases(5, F))
    assert rel_rms(wav.cpu().numpy()[0], ref) < WAV_RTOL
    # and without a speaker id the reference adds no embedding: not the speaker fixture's output
    wav0, _ = m.synthesize_native([z["ids"]], ap, seed=5)
    assert not torch.equal(wav0, wav)


BN_CASES = ["t2bn_fwdmask_L24", "t2bn_fwdmask_L40"]


def _bn_model(**kw):
    t2 = load_pkg("tacotron2")
    fl = golden_flags(golden(BN_CASES[0]))
    m = t2.Tacotron2(130, 0, r=1, attn_win=fl["attn_win"], attn_norm=fl["attn_norm"], forward_attn=fl["forward_attn"],
                     trans_agent=fl["trans_agent"], forward_attn_mask=fl["forward_attn_mask"],
                     location_attn=fl["location_attn"], prenet_type="bn", **kw)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in weights_mod().tacotron2_weights(0, prenet_bn=True).items()})
    m.decoder.max_decoder_steps = fl["max_decoder_steps"]
    return m.cuda().eval()


@pytest.mark.parametrize("case", BN_CASES)
def test_prenet_bn_inference_vs_reference(case):
    """prenet_type "bn" at batch 1 (the resident decoder: BatchNorm folded into the prenet rows,
    prenet-2 bias per XCD row, prenet-1 bias in the folded mel rows) against the reference run."""
    z = golden(case)
    m = _bn_model()
    mel, mel_post, align, stop = m.inference(torch.from_numpy(z["ids"])[None])
    assert mel.shape == (1,) + z["mel"].shape
    np.testing.assert_array_equal(align[0].cpu().numpy().argmax(1), z["align"].argmax(1))
    np.testing.assert_array_equal(stop[0, :, 0].cpu().numpy() > 0.5, z["stop"] > 0.5)
    assert rel_rms(mel[0].cpu().numpy(), z["mel"]) < MEL_RTOL
    assert rel_rms(mel_post[0].cpu().numpy(), z["mel_post"]) < MEL_RTOL


@pytest.mark.parametrize("B", [2, 20])
def test_prenet_bn_batch_vs_reference(B):
    """prenet_type "bn" through the multi-launch batched step (prenet GEMM biases; B = 20 also the
    fragment-mirror GEMMs) from the reference's encoder outputs, alternating the two fixtures."""
    zs = [golden(BN_CASES[b % 2]) for b in range(B)]
    m = _bn_model(max_batch=max(B, 2))
    Lmax = max(len(z["ids"]) for z in zs)
    enc = torch.zeros(B, Lmax, 512)
    for b, z in enumerate(zs):
        enc[b, :len(z["ids"])] = torch.from_numpy(z["enc"])
    out = m.inference_batch(None, enc=enc.cuda(), lens=[len(z["ids"]) for z in zs])
    for b, z in enumerate(zs):
        _check_decoder(out, b, z)


@pytest.mark.parametrize("B", [3, 20])
def test_location_attention_batch_vs_reference(B):
    """Location-sensitive attention with forward attention and the transition agent (the multi-launch
    path: energies with the location term as query-launch partials, the split attention launch with
    the next step's location features) in a batch of 3 (row-major GEMM inputs) and of 20 (fragment
    mirrors, written slice by slice), against the reference run."""
    z = golden("t2_loc_fwd_ta_L24")
    m = _model(golden_flags(z))
    L = len(z["ids"])
    enc = torch.from_numpy(z["enc"])[None].repeat(B, 1, 1).cuda()
    out = m.inference_batch(None, enc=enc, lens=[L] * B)
    for b in range(B):
        _check_decoder(out, b, z)
