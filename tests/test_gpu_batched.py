"""GPU parity of the batched configurations (BASELINE configs[2], [3], [4]) on the paths they
actually take: at B * Fmax > 1024 Griffin-Lim runs the unfused batched loop (gl_ola_kernel +
gl_iter_kernel<false, false> per iteration), which the small-batch tests never reach.  Each test
asserts the path it took (launch count) and checks sentences against the oracle chain at the
metric's 60 iterations (waveform relative RMS 1e-4, frame counts exact)."""
import numpy as np
import pytest
import torch

from conftest import golden, golden_flags, load_pkg, rel_rms, weights_mod
from oracle.griffin_lim_oracle import AudioOracle, device_phase_u
from oracle.tacotron2_oracle import Tacotron2Oracle

pytestmark = pytest.mark.gpu
WAV_RTOL = 1e-4
MEL_RTOL = 4e-6  # model half: 10x the measured worst case (profiles/r05f_parity_report.jsonl)


def _t2(max_batch=64, **over):
    gu = load_pkg("generic_utils")
    cfg = gu.default_config("config_tacotron2.json")
    cfg.forward_attn_mask = True  # synthesize.py:86
    cfg.update(over)
    m = gu.setup_model(130, cfg, max_batch=max_batch, max_len=256).cuda().eval()
    return cfg, m


def test_config2_batch64_unfused_griffin_lim_vs_oracle(audio_cfg):
    """configs[2]: B=64, L ~ U{60..160} (seed 2), synthesize_batch with the reference's numpy
    phases (one np.random.rand(1025, T_b) per sentence in batch order) at 60 iterations; the
    shortest and the longest sentence's waveforms vs the oracle GL on the same mel_post."""
    w = weights_mod()
    lens = w.synthetic_lengths(64, 2)
    ids = [w.synthetic_ids(int(L), 100 + b) for b, L in enumerate(lens)]
    cfg, m = _t2()
    ap = load_pkg("audio").AudioProcessor(**audio_cfg)
    np.random.seed(21)
    wavs, info = load_pkg("synthesis").synthesize_batch(m, ap, ids, phase="numpy", keep_outputs=True)
    frames = info["frames"]
    assert frames == [2 * int(L) + 22 for L in lens]
    assert 64 * max(frames) > 1024 and info["gl_iterations"] == 2 * 60, "not the unfused batched GL loop"
    np.random.seed(21)
    pus = [np.random.rand(1025, T) for T in frames]
    o = AudioOracle(**audio_cfg)
    for b in (int(np.argmin(lens)), int(np.argmax(lens))):
        T = frames[b]
        mel_post = info["mel_post"][b, :T].cpu().numpy()
        ref = o.inv_mel_spectrogram(mel_post.T, pus[b])
        assert wavs[b].shape == ref.shape
        assert rel_rms(wavs[b], ref) < WAV_RTOL, b


def test_config3_rank_share_sharded_vs_oracle_chain(audio_cfg):
    """configs[3]'s per-rank workload: rank 0's LPT share (64 sentences) of the 512-sentence seed-3
    job, through sharding.synthesize_sharded on a 1-rank RCCL group; two sentences (shortest,
    longest) vs the oracle chain ids -> Tacotron2 -> GL 60 with the device phases restated, stage by
    stage at 1e-4 (mel_post; GL of that mel_post) and compounded at 1e-3."""
    import torch.distributed as dist
    sh = load_pkg("sharding")
    w = weights_mod()
    lens = w.synthetic_lengths(512, 3)
    all_ids = [w.synthetic_ids(int(L), 100 + b) for b, L in enumerate(lens)]
    costs = [sh.sentence_cost(len(x), 1000) for x in all_ids]
    mine = sh.lpt_partition(costs, 8, capacity=64)[0]
    ids = [all_ids[i] for i in mine]
    assert len(ids) == 64
    cfg, m = _t2()
    ap = load_pkg("audio").AudioProcessor(**audio_cfg)
    store = dist.TCPStore("127.0.0.1", 0, 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1)
    try:
        pcm, info = sh.synthesize_sharded(m, ap, ids, seed=40)
    finally:
        dist.destroy_process_group()
    frames = info["frames"]
    assert frames == [2 * len(x) + 22 for x in ids]
    assert info["gl_iterations"] == 2 * 60, "not the unfused batched GL loop"
    n = [ap.hop_length * (T - 1) for T in frames]
    assert pcm.dtype == np.int16 and len(pcm) == sum(n) + 10000 * len(ids)
    fl = golden_flags(golden("t2_fwdmask_L100"))
    o = Tacotron2Oracle(w.tacotron2_weights(0), dtype=np.float32, **fl)
    ao = AudioOracle(**audio_cfg)
    Ls = [len(x) for x in ids]
    for b in (int(np.argmin(Ls)), int(np.argmax(Ls))):
        T = frames[b]
        ref = o.inference(ids[b])
        assert ref["mel"].shape[0] == T
        # stage by stage at the north_star tolerance: the model's mel_post, then Griffin-Lim on it
        mel_post = info["mel_post"][b, :T].cpu().numpy()
        assert rel_rms(mel_post, ref["mel_post"]) < MEL_RTOL, b
        pu = device_phase_u(40, b, T)
        got = info["wavs"][b].cpu().numpy()
        gl_ref = ao.inv_mel_spectrogram(mel_post.T, pu)
        assert got.shape == gl_ref.shape
        assert rel_rms(got, gl_ref) < WAV_RTOL, b
        # the compounded chain: Griffin-Lim amplifies the model's ~1e-7 fp32 reduction-order
        # differences (60 iterations, phase retrieval is unstable where |X| ~ 0) by ~10^3 on the
        # longest sentences, so the end-to-end waveform is held to 1e-3 (measured 1.5e-4 at T=342)
        wav_ref = ao.inv_mel_spectrogram(ref["mel_post"].T, pu)
        assert rel_rms(got, wav_ref) < 1e-3, b


def test_config4_gst_batch32_linear_unfused_griffin_lim_vs_oracle():
    """configs[4] shape on the linear-spectrogram GL: TacotronGST B=32 (L ~ U{60..160}, seed 4,
    speakers b mod 4, style mel seed 4), decoder cap lowered to 60 steps (300 frames per sentence,
    so the CPU oracle stays in seconds; B * Fmax = 9600 > 1024 keeps the unfused loop), GL 60 with
    numpy phases; two sentences vs the oracle's inv_spectrogram of the GPU linear output."""
    w = weights_mod()
    gu = load_pkg("generic_utils")
    audio = load_pkg("audio")
    cfg = gu.default_config("config_tacotron_gst.json")
    m = gu.setup_model(130, 4, cfg, max_batch=32, max_len=256).cuda().eval()
    m.decoder.max_decoder_steps = 60
    lens = w.synthetic_lengths(32, 4)
    ids = [w.synthetic_ids(int(L), 200 + b) for b, L in enumerate(lens)]
    rng = np.random.Generator(np.random.PCG64(4))
    style = torch.from_numpy(rng.uniform(0, 1, size=(32, 200, 80)).astype(np.float32)).cuda()
    spk = [b % 4 for b in range(32)]
    out = m.inference_batch(ids, speaker_ids=spk, style_mel=style)
    frames = out["frames"]
    ap = audio.AudioProcessor(**cfg.audio)
    assert ap.griffin_lim_iters == 60
    np.random.seed(31)
    pu = np.zeros((32, 1025, max(frames)))
    for b, T in enumerate(frames):
        pu[b, :, :T] = np.random.rand(1025, T)
    wav = ap.griffin_lim_batch(out["linear"], frames, mode=audio._native.TTS_GL_FROM_LINEAR, phase_u=pu)
    assert 32 * max(frames) > 1024 and ap.last_gl_timing()["gl_iterations"] == 2 * 60
    wav = wav.cpu().numpy()
    o = AudioOracle(**cfg.audio)
    for b in (0, 13):
        T = frames[b]
        lin = out["linear"][b, :T].cpu().numpy()
        ref = o.inv_spectrogram(lin.T, pu[b, :, :T])
        nb = ap.hop_length * (T - 1)
        assert rel_rms(wav[b, :nb], ref) < WAV_RTOL, b
        assert np.all(wav[b, nb:] == 0)


def test_config4_gst_batch32_full_cap_linear_griffin_lim_vs_oracle():
    """configs[4] exactly as benched: TacotronGST B=32 at the real 500-step cap (r=5: up to 2505
    frames, the length where the bench spends 88% of its Griffin-Lim frames, beyond anything the
    60-step test reaches), linear GL 60 iterations with device phases (seed 17).  The longest
    sentence's waveform vs the oracle's inv_spectrogram of the GPU linear output on the restated
    device phases at 1e-4; every sentence finite and zero past its own length."""
    w = weights_mod()
    gu = load_pkg("generic_utils")
    audio = load_pkg("audio")
    cfg = gu.default_config("config_tacotron_gst.json")
    m = gu.setup_model(130, 4, cfg, max_batch=32, max_len=256).cuda().eval()
    assert m.decoder.max_decoder_steps == 500  # layers/tacotron.py:278
    lens = w.synthetic_lengths(32, 4)
    ids = [w.synthetic_ids(int(L), 200 + b) for b, L in enumerate(lens)]
    rng = np.random.Generator(np.random.PCG64(4))
    style = torch.from_numpy(rng.uniform(0, 1, size=(32, 200, 80)).astype(np.float32)).cuda()
    out = m.inference_batch(ids, speaker_ids=[b % 4 for b in range(32)], style_mel=style)
    frames = out["frames"]
    assert max(frames) > 2048
    ap = audio.AudioProcessor(**cfg.audio)
    wav = ap.griffin_lim_batch(out["linear"], frames, mode=audio._native.TTS_GL_FROM_LINEAR, seed=17)
    assert ap.last_gl_path() == "unfused" and ap.last_gl_timing()["gl_iterations"] == 2 * 60
    wav = wav.cpu().numpy()
    assert np.isfinite(wav).all()
    for b, T in enumerate(frames):
        assert np.all(wav[b, ap.hop_length * (T - 1):] == 0), b
    b = int(np.argmax(frames))
    T = frames[b]
    lin = out["linear"][b, :T].cpu().numpy()
    ref = AudioOracle(**cfg.audio).inv_spectrogram(lin.T, device_phase_u(17, b, T))
    nb = ap.hop_length * (T - 1)
    assert rel_rms(wav[b, :nb], ref) < WAV_RTOL, (b, T)


@pytest.mark.parametrize("txt,sens_ref,kind", [
    ("It took me quite a long time. Dr. Smith spoke! Ok? Then we left.",
     ["It took me quite a long time.", "Dr. Smith spoke!", "Ok?", "Then we left."], 2),
    ("It took me quite a long time. Dr. Smith spoke! Then we left.",
     ["It took me quite a long time.", "Dr. Smith spoke!", "Then we left."], 2),
    ("It took me quite a long time.", ["It took me quite a long time."], 1)])
def test_synthesizer_tts_vs_oracle_chain(audio_cfg, txt, sens_ref, kind):
    """Synthesizer.tts (server/synthesizer.py:128-162) on a multi-sentence text with the reference's
    numpy phases: split, drop len < 3, per-sentence Tacotron2 (cap 3000) + GL in order, 10 000-zero
    gaps, one global peak -> int16, vs the oracle chain doing exactly that one sentence at a time.
    Requests of several sentences decode on the resident batch decoder in one tts_synth_run (kind 2),
    one sentence on the batch-1 resident decoder (kind 1)."""
    import scipy.io.wavfile
    text = load_pkg("text")
    synth = load_pkg("synthesis")
    cfg, m = _t2(max_batch=8)
    a = {**audio_cfg, "griffin_lim_iters": 20}
    ap = load_pkg("audio").AudioProcessor(**a)
    adapter = lambda s: text.text_to_sequence(s, ["basic_cleaners"])  # noqa: E731
    s = synth.Synthesizer(m, ap, cfg, input_adapter=adapter)
    sens = s.sentences(txt)
    assert sens == sens_ref
    np.random.seed(77)
    buf = s.tts(txt)
    assert m.last_timing["resident_kind"] == kind
    buf.seek(0)
    sr, pcm = scipy.io.wavfile.read(buf)
    assert sr == 22050 and pcm.dtype == np.int16
    np.random.seed(77)
    fl = golden_flags(golden("t2_fwdmask_L100"))
    o = Tacotron2Oracle(weights_mod().tacotron2_weights(0), dtype=np.float32, max_decoder_steps=3000,
                        **{k: v for k, v in fl.items() if k != "max_decoder_steps"})
    ao = AudioOracle(**a)
    wavs = []
    refs = [o.inference(np.asarray(adapter(x))) for x in sens]
    for ref in refs:  # phases drawn sentence by sentence in order, as the reference's loop does
        wavs += list(ao.inv_mel_spectrogram(ref["mel_post"].T)) + [0] * 10000
    ref_pcm = AudioOracle.wav_to_int16(np.array(wavs))
    assert pcm.shape == ref_pcm.shape
    assert np.abs(pcm.astype(np.int32) - ref_pcm).max() <= 2


@pytest.mark.parametrize("truncated", [False, True])
def test_tacotron2_synthesis_both_modes(audio_cfg, truncated):
    """synthesis() on Tacotron2 (utils/synthesis.py:78-124): the 5-tuple for both values of
    truncated (inference / inference_truncated -> parse_outputs -> inv_mel_spectrogram), vs the
    reference's model outputs and the oracle GL with the same numpy phases."""
    z = golden("t2_fwdmask_L12")
    cfg, m = _t2(max_batch=4)
    a = {**audio_cfg, "griffin_lim_iters": 10}
    ap = load_pkg("audio").AudioProcessor(**a)
    np.random.seed(5)
    wav, alignment, dec, post, stop = load_pkg("synthesis").synthesis(m, z["ids"], cfg, True, ap,
                                                                       truncated=truncated)
    assert post.shape == z["mel_post"].shape and dec.shape == z["mel"].shape
    assert alignment.shape == z["align"].shape and tuple(stop.shape) == (1, z["mel"].shape[0], 1)
    assert rel_rms(post, z["mel_post"]) < MEL_RTOL and rel_rms(dec, z["mel"]) < MEL_RTOL
    np.testing.assert_array_equal(alignment.argmax(1), z["align"].argmax(1))
    np.random.seed(5)
    ref = AudioOracle(**a).inv_mel_spectrogram(z["mel_post"].T)
    assert wav.shape == ref.shape and rel_rms(wav, ref) < 1e-4


def test_griffin_lim_wave_kernel_ragged_vs_oracle(audio_cfg, monkeypatch):
    """The one-wave-per-frame iteration kernel (gl_iter_wave_kernel, the batched default) on a
    ragged batch whose B * Fmax keeps the unfused loop: sentences of 2, 3 and 5 frames (every
    frame's STFT input reflected at both ends), mid-length and long ones; each sentence vs the
    oracle at 60 iterations (1e-4) and vs the 256-thread block kernel (TTS_GL_WAVE=0) on the same
    phases."""
    audio = load_pkg("audio")
    o = AudioOracle(**audio_cfg)
    rng = np.random.Generator(np.random.PCG64(11))
    Fs = [2, 3, 5, 150, 33, 220, 64, 7]
    Fmax = max(Fs)
    assert len(Fs) * Fmax > 1024
    mel = np.zeros((len(Fs), Fmax, 80), np.float32)
    pu = np.zeros((len(Fs), 1025, Fmax))
    for b, F in enumerate(Fs):
        mel[b, :F] = rng.uniform(0, 1, size=(F, 80))
        pu[b, :, :F] = rng.uniform(0, 1, size=(1025, F))
    mel_d = torch.from_numpy(mel).cuda()
    ap = audio.AudioProcessor(**audio_cfg)
    wav = ap.griffin_lim_batch(mel_d, Fs, phase_u=pu).cpu().numpy()
    assert ap.last_gl_path() == "unfused"
    monkeypatch.setenv("TTS_GL_WAVE", "0")
    ap_block = audio.AudioProcessor(**audio_cfg)
    wav_block = ap_block.griffin_lim_batch(mel_d, Fs, phase_u=pu).cpu().numpy()
    for b, F in enumerate(Fs):
        n = ap.hop_length * (F - 1)
        ref = o.inv_mel_spectrogram(mel[b, :F].T, pu[b, :, :F])
        assert rel_rms(wav[b, :n], ref) < WAV_RTOL, (b, F)
        assert rel_rms(wav[b, :n], wav_block[b, :n]) < WAV_RTOL, (b, F)
        assert np.all(wav[b, n:] == 0)


def test_overlap_add_launch_bitwise_vs_in_kernel_gather(audio_cfg, monkeypatch):
    """gl_ola_kernel takes the window sum-square of samples with every contributor present from a
    per-(u mod hop) table summed on the host; the fused block kernel sums win^2 per sample itself
    (ola_sample_unrolled). With the block kernel on both sides (TTS_GL_WAVE=0) the unfused loop
    (overlap-add launch + iteration launch) and the forced in-kernel gather (TTS_GL_FUSED=1) must
    give bitwise the same waveform on a ragged batch, edges and reflected short sentences included."""
    audio = load_pkg("audio")
    rng = np.random.Generator(np.random.PCG64(12))
    Fs = [2, 4, 6, 300, 41, 290, 9, 130]
    Fmax = max(Fs)
    mel = np.zeros((len(Fs), Fmax, 80), np.float32)
    pu = np.zeros((len(Fs), 1025, Fmax))
    for b, F in enumerate(Fs):
        mel[b, :F] = rng.uniform(0, 1, size=(F, 80))
        pu[b, :, :F] = rng.uniform(0, 1, size=(1025, F))
    mel_d = torch.from_numpy(mel).cuda()
    monkeypatch.setenv("TTS_GL_WAVE", "0")
    ap = audio.AudioProcessor(**audio_cfg)
    wav = ap.griffin_lim_batch(mel_d, Fs, phase_u=pu).cpu().numpy()
    assert ap.last_gl_path() == "unfused"
    monkeypatch.setenv("TTS_GL_FUSED", "1")
    ap_f = audio.AudioProcessor(**audio_cfg)
    wav_f = ap_f.griffin_lim_batch(mel_d, Fs, phase_u=pu).cpu().numpy()
    assert ap_f.last_gl_path() == "fused"
    assert np.array_equal(wav, wav_f)


def test_griffin_lim_wave_kernel_initial_istft_vs_oracle(audio_cfg, monkeypatch):
    """The batched loops' initial iSTFT on the one-wave-per-frame layout (gl_iter_wave_kernel<true>):
    with zero iterations the waveform is that launch's output alone (plus the overlap-add), so it is
    held much tighter than after 60 iterations (no Griffin-Lim amplification): vs the oracle's
    istft(|S| exp(2 pi i U)) and vs the 256-thread block kernels (TTS_GL_WAVE=0)."""
    audio = load_pkg("audio")
    cfg = {**audio_cfg, "griffin_lim_iters": 0}
    o = AudioOracle(**cfg)
    rng = np.random.Generator(np.random.PCG64(13))
    Fs = [3, 150, 33, 220, 64, 7]
    Fmax = max(Fs)
    assert len(Fs) * Fmax > 1024  # the unfused (batched) loop
    mel = np.zeros((len(Fs), Fmax, 80), np.float32)
    pu = np.zeros((len(Fs), 1025, Fmax))
    for b, F in enumerate(Fs):
        mel[b, :F] = rng.uniform(0, 1, size=(F, 80))
        pu[b, :, :F] = rng.uniform(0, 1, size=(1025, F))
    mel_d = torch.from_numpy(mel).cuda()
    ap = audio.AudioProcessor(**cfg)
    wav = ap.griffin_lim_batch(mel_d, Fs, phase_u=pu).cpu().numpy()
    assert ap.last_gl_path() == "unfused"
    monkeypatch.setenv("TTS_GL_WAVE", "0")
    wav_block = audio.AudioProcessor(**cfg).griffin_lim_batch(mel_d, Fs, phase_u=pu).cpu().numpy()
    for b, F in enumerate(Fs):
        n = ap.hop_length * (F - 1)
        ref = o.inv_mel_spectrogram(mel[b, :F].T, pu[b, :, :F])
        assert rel_rms(wav[b, :n], ref) < 1e-6, (b, F)
        assert rel_rms(wav[b, :n], wav_block[b, :n]) < 1e-6, (b, F)
