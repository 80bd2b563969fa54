#!/usr/bin/env python3
"""Headline benchmark: mel-frames/s and RTF of Tacotron2 + 60-iteration Griffin-Lim on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--L 100] [--iters 60]

A step = one pass of the synthesis hot path over one batch of synthetic sentences per rank:
ids (already in HBM) -> encoder -> HIP decoder loop -> HIP postnet -> HIP Griffin-Lim (60 iters,
inverse pre-emphasis) -> waveforms in HBM; with N > 1 ranks the finished waveforms are gathered to
rank 0 over RCCL (the only collective: sentences are independent).  Weak scaling:
every rank synthesises --batch sentences per step.

Default workload = BASELINE.json configs[1]: one LJSpeech-length sentence (L=100 ids, seed 1,
-> 222 frames), config_tacotron2.json + forward_attn_mask (synthesize.py:86), random-init weights
from the deterministic generator (seed 0), GL 60 iterations.  ``--model gst`` measures configs[4]
instead: TacotronGST (config_tacotron_gst.json, 4 speakers, speaker b mod 4), B=32 sentences per
GPU with L ~ U{60..160} (seed 4), style mel [B, 200, 80] ~ U[0,1) (seed 4), linear-spectrogram GL.

Prints ONE JSON line on rank 0 (keys per the driver contract, plus roofline / cpu_baseline).
"""
from __future__ import annotations

import argparse
import glob
import importlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
pkg = importlib.import_module("your-voice-tts_amd")
t2mod = importlib.import_module("your-voice-tts_amd.tacotron2")
audiomod = importlib.import_module("your-voice-tts_amd.audio")
weights = importlib.import_module("your-voice-tts_amd.weights")
gu = importlib.import_module("your-voice-tts_amd.generic_utils")
sharding = importlib.import_module("your-voice-tts_amd.sharding")

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)
FP32_MFMA_PEAK_TF = 157.3  # dense fp32 MFMA peak (same table)
# one hand-off edge of the resident decoder in isolation (tools/microbench/edge.hip, one 16-byte
# granule pair per lane; device-wide 1024 granules on 8 waves, XCD-local 256 on 4 waves), the best
# over first-poll delays (round 6, profiles/r06_edge_floor.log: device-wide 1.61 us polling at once,
# 0.98 with a ~0.36 us delay; XCD-local 0.76, no delay; round 4 had measured 1.60 / 0.47)
EDGE_DEVICE_US = 0.98
EDGE_XCD_US = 0.76
FP64_VECTOR_PEAK_TF = 78.6  # fp64 vector FMA peak (same table)
# one GL frame-iteration: forward + inverse 1024-point complex FFT (5 N log2 N each) plus the
# real-FFT split / merge and the phase projection (~20 flops per bin each way)
GL_FLOPS_PER_FRAME_ITER = 2 * 5 * 1024 * 10 + 2 * 20 * 1025
POSTNET_FLOP_PER_FRAME = 2 * 5 * (80 * 512 + 3 * 512 * 512 + 512 * 80)
GL_BYTES_PER_FRAME_ITER = 4 * 1025 + 2 * 4 * 275                        # 6300 B


def kernel_algorithmic(name, B, L, frames_total, r=1):
    """(kind, algorithmic bytes or flops per launch) for each timed kernel."""
    nm = 80 * r
    by = {
        "prenet2": 4 * (256 * 256 + B * (256 + 256)),
        "att_lstm": 4 * (4096 * 1792 + B * (1792 + 3 * 1024)),
        # query_layer GEMV + energy partials: W_q, h, P (128 per position) in; q and 8 partials out
        "query": 4 * (128 * 1024 + B * (1024 + 128 + L * (128 + 8))),
        # energies from partials, forward attention: 8 partials + alpha[j], alpha[j-1] in, alpha and
        # the alignment row out; the context touches only the <= 5 surviving encoder rows
        "attention": 4 * B * (L * (8 + 2 + 2) + 5 * 512 + 512),
        "dec_lstm": 4 * (4096 * 2560 + B * (2560 + 3 * 1024)),
        # fused mel projection (nm rows) + folded prenet L1 (256 rows) + folded stopnet (1 row)
        "mel_fused": 4 * ((nm + 257) * 1536 + B * (1536 + nm + 256 + 1)),
        "gl_iter": GL_BYTES_PER_FRAME_ITER * frames_total,
    }
    return ("hbm", by[name])


def decoder_step_algorithmic(B, L):
    """algorithmic bytes of one decoder step at batch B (weights once per batch-step,
    inputs + processed inputs, state / outputs) — 72.99 MB at B=1, L=100."""
    return 4 * 18183458 + 4 * B * L * 640 + 4 * B * (3 * 1024 + 2 * 1024 + 512 + 80 + L)


def decoder_step_flops(L):
    """fp32 flops of one sentence-step (2 x 18 166 864 weight MACs + the attention's
    1 280 per encoder position) — 36.46 MFLOP at L=100."""
    return 2 * 18166864 + 1280 * L


def kernel_algorithmic_gst(name, B, L, frames_total, r=5):
    """Algorithmic bytes per launch of the TacotronGST decoder-step kernels (weights once per batch
    step + per-sentence activations) and of the GL iteration."""
    nm = 80 * r
    by = {
        "prenet2": 4 * (128 * 256 + B * (256 + 128)),
        "att_gru": 4 * (3 * 256 * 640 + B * (640 + 2 * 256)),
        "query": 4 * (128 * 256 + B * (256 + 128)),
        "attention": 4 * B * (L * (128 + 256 + 3) + 128 + 256),
        "proj": 4 * (256 * 512 + B * (512 + 256)),
        "dec_gru1": 4 * (3 * 256 * 512 + B * (512 + 3 * 256)),
        "dec_gru2": 4 * (3 * 256 * 512 + B * (512 + 3 * 256)),
        "mel": 4 * (nm * 256 + B * (256 + 2 * nm)),
        "pre1_stop": 4 * ((256 + 1) * (nm + 256) + B * (nm + 256 + 257)),
        "gl_iter": GL_BYTES_PER_FRAME_ITER * frames_total,
    }
    return ("hbm", by[name])


def build(args, device):
    if args.model == "gst":
        cfg = gu.default_config("config_tacotron_gst.json")
        model = gu.setup_model(130, 4, cfg, max_batch=max(args.batch, 1), max_len=256)
        model.load_state_dict({k: torch.from_numpy(v) for k, v in weights.tacotron_gst_weights(0, num_speakers=4).items()})
        model.cuda().eval()
        audio = dict(cfg.audio)
        audio["griffin_lim_iters"] = args.iters
        return cfg, model, audiomod.AudioProcessor(**audio)
    cfg = gu.default_config("config_tacotron2.json")
    cfg.forward_attn_mask = True  # synthesize.py:86
    model = gu.setup_model(130, cfg, max_batch=max(args.batch, 1), max_len=max(args.L, 256))
    model.load_state_dict({k: torch.from_numpy(v) for k, v in weights.tacotron2_weights(0).items()})
    model.cuda().eval()
    audio = dict(cfg.audio)
    audio["griffin_lim_iters"] = args.iters
    ap = audiomod.AudioProcessor(**audio)
    return cfg, model, ap


def build_server_model(args, max_batch=1):
    """Synthesizer.tts()'s model (server/synthesizer.py:46-66): config_tacotron2.json as it is (forward
    attention, sigmoid, eval mask OFF) with the 3000-step decoder cap; same generator weights."""
    cfg = gu.default_config("config_tacotron2.json")
    model = gu.setup_model(130, cfg, max_batch=max_batch, max_len=max(args.L, 256))
    model.load_state_dict({k: torch.from_numpy(v) for k, v in weights.tacotron2_weights(0).items()})
    model.decoder.max_decoder_steps = 3000
    return model.cuda().eval()


def make_job(args, world, rank, max_steps, model=None, batch=None, lengths=None, seed=None):
    """The whole job's sentences (world x batch) and this rank's LPT share (sharding.py)."""
    model = args.model if model is None else model
    batch = args.batch if batch is None else batch
    lengths = args.lengths if lengths is None else lengths
    n = world * batch
    if model == "gst":
        # configs[4]: L ~ U{60..160} (seed 4); every sentence costs up to the 500-step cap
        lens = weights.synthetic_lengths(n, 4)
        ids = [weights.synthetic_ids(int(L), 200 + b) for b, L in enumerate(lens)]
        mine = sharding.lpt_partition([len(x) for x in ids], world, capacity=batch)[rank]
        return ids, mine
    if lengths == "fixed":
        ids = [weights.synthetic_ids(args.L, 1) for _ in range(n)]  # configs[1]: L=100, seed 1
    else:
        # configs[2] (B=64, seed 2) on one GPU; configs[3] (B=512 over 8 GPUs, seed 3) otherwise
        if seed is None:
            seed = 2 if world == 1 else 3
        lens = weights.synthetic_lengths(n, seed)
        ids = [weights.synthetic_ids(int(L), 100 + b) for b, L in enumerate(lens)]
    costs = [sharding.sentence_cost(len(x), max_steps) for x in ids]
    mine = sharding.lpt_partition(costs, world, capacity=batch)[rank]
    return ids, mine


CONFIGS3_WORLD = 8  # BASELINE configs[3]: 512 sentences over 8 GPUs, 64 per rank


def configs3_share(args, max_steps):
    """Rank 0's LPT share of the configs[3] job (512 seed-3 sentences over 8 ranks, 64 each): the
    per-rank workload of the driver's 8-GPU run, which the N=1 line times on one GPU too."""
    return make_job(args, CONFIGS3_WORLD, 0, max_steps, model="tacotron2", batch=64, lengths="uniform", seed=3)


_STYLE = {}


def gst_inputs(n, device):
    """configs[4] style mels [n, 200, 80] ~ U[0,1) (seed 4) in HBM and speakers b mod 4."""
    if n not in _STYLE:
        rng = np.random.Generator(np.random.PCG64(4))
        _STYLE[n] = torch.from_numpy(rng.uniform(0, 1, size=(n, 200, 80)).astype(np.float32)).to(device)
    return _STYLE[n], [b % 4 for b in range(n)]


@torch.no_grad()
def run_step(model, ap, ids, mine, world, seed):
    if hasattr(model, "linear_dim"):  # TacotronGST: linear spectrogram -> inv_spectrogram GL
        style, spk = gst_inputs(len(ids), model.device)
        sel = torch.as_tensor(mine, dtype=torch.long, device=model.device)
        out = model.inference_batch([ids[i] for i in mine], speaker_ids=[spk[i] for i in mine],
                                    style_mel=style.index_select(0, sel))
        wav = ap.griffin_lim_batch(out["linear"], out["frames"], mode=audiomod._native.TTS_GL_FROM_LINEAR, seed=seed)
    else:
        # ids -> wav in one native call (tts_synth_run): the same stage entry points as
        # inference_batch + griffin_lim_batch, without the host round trips between them
        wav, frames = model.synthesize_native([ids[i] for i in mine], ap, seed=seed, sync=False)
        out = dict(frames=frames)
    if world > 1:
        # finished waveforms only, gather-v to rank 0 over RCCL (point-to-point, one link per peer)
        rows = [wav[k, :ap.hop_length * (T - 1)] for k, T in enumerate(out["frames"])]
        sharding.gather_waveforms(rows, mine, len(ids))
    return out["frames"], wav


SERVER_SENTENCES = ["It took me quite a long time to develop a voice.", "Now that I have it I am not going to be silent.",
                    "Dr. Smith spoke to the crowd for an hour!", "Then we all went home?"]


def synthesizer_tts_wall(args, ap, gpu_ms_per_sentence):
    """The drop-in the reference's server runs, timed end to end (VERDICT r5 missing 1):
    Synthesizer.tts(text) -> BytesIO (split, ids, decode, Griffin-Lim with numpy's phase stream,
    10 000-zero join, int16 save_wav) at the server configuration (config_tacotron2.json, mask off,
    3000-step cap), for a 1- and a 4-sentence request.  Each sentence maps to synthetic ids of length
    args.L (the text front-end is not on the path).  Wall clock on the host, numpy seeded per request."""
    synth = importlib.import_module("your-voice-tts_amd.synthesis")
    sm = build_server_model(args, max_batch=4)
    cfg = gu.default_config("config_tacotron2.json")
    table = {sen: weights.synthetic_ids(args.L, 1 + k) for k, sen in enumerate(SERVER_SENTENCES)}
    s = synth.Synthesizer(sm, ap, cfg, input_adapter=lambda sen: table[sen])
    out = {}
    for n, reps in ((1, 3), (4, 2)):
        text = " ".join(SERVER_SENTENCES[:n])
        assert len(s.sentences(text)) == n
        np.random.seed(0)
        s.tts(text)  # warm (handles, graphs, buffers)
        walls = []
        for r in range(reps):
            np.random.seed(r)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            buf = s.tts(text)
            walls.append(1000 * (time.perf_counter() - t0))
        rec = dict(sentences=n, wall_ms=float(np.median(walls)), wall_ms_runs=walls, wav_bytes=len(buf.getvalue()),
                   decoder="resident" if sm.last_timing.get("resident") else "multi-launch",
                   dispatch="serial one-call (tts_synth_run)" if n <= synth.SERIAL_RESIDENT_MAX else "batch")
        if n == 1 and gpu_ms_per_sentence:
            rec["gpu_ms"] = gpu_ms_per_sentence
            rec["wall_over_gpu"] = rec["wall_ms"] / gpu_ms_per_sentence
        out[f"{n}_sentence"] = rec
    out["note"] = ("Synthesizer.tts(text) -> BytesIO, host work included (phases drawn from numpy's MT19937 stream on "
                   "the device, device int16 join); gpu_ms = synthesizer_config_1rank ms_per_step (the same "
                   "sentence's GPU time through the one-call path, back to back)")
    del s, sm
    return out


def collect_status(model):
    """The timed loop pipelines tts_synth_run (sync=False): the LAST call's Griffin-Lim status is
    only collected by tts_synth_sync (a device synchronize does not read it).  Raise if it failed,
    so a timed-out persistent loop can never hide inside a published measurement."""
    if hasattr(model, "synth_sync"):
        model.synth_sync()


def _cpu_model():
    """lscpu's model name and the logical CPUs this process may run on."""
    name = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                name = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except Exception:
        avail = os.cpu_count()
    return f"{name} ({avail} logical CPUs available to this process)"


def _threads():
    try:
        from threadpoolctl import threadpool_info
        return max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        return 1


def _physical_cores():
    """(threads, how): physical cores this process may use — distinct (package, core) pairs of its
    CPU affinity set, capped by the cgroup CPU quota and by OMP_NUM_THREADS (the GPU box sets it to
    its per-GPU CPU share)."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except Exception:
        cpus = list(range(os.cpu_count() or 1))
    cores = set()
    for c in cpus:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            cores.add((open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip()))
        except OSError:
            cores.add(("?", str(c)))
    n = len(cores)
    how = [f"{n} physical cores in the affinity set ({len(cpus)} logical)"]
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            lim = max(1, int(int(q) / int(per)))
            how.append(f"cgroup quota {lim} CPUs")
            n = min(n, lim)
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        how.append(f"OMP_NUM_THREADS={omp}")
        n = min(n, int(omp))
    return max(1, n), "; ".join(how)


def _port_over_reference(section="model"):
    """The committed CPU port vs reference timing (tools/cpu_port_vs_reference.py, build container:
    the reference cannot run on the GPU box); section "model" (Tacotron2) or "gst_model"."""
    for p in sorted(glob.glob(os.path.join(REPO, "profiles", "cpu_port_vs_reference_r*.json")), reverse=True):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if section not in d:
            continue
        out = {f"model_{k}": round(v["port_over_reference"], 3) for k, v in d[section].items()}
        if "griffin_lim" in d and section == "model":
            out["griffin_lim_60"] = round(d["griffin_lim"]["port_over_reference"], 3)
        out["source"] = os.path.relpath(p, REPO) + " (" + d.get("cpu_model", "?") + ")"
        return out
    return None


def cpu_baseline_gst(args):
    """The reference's CPU path for configs[4] restated on the host: TacotronGST as torch-CPU modules
    (oracle/tacotron_torch.py, the reference's module tree and op order) on the process's physical
    cores + the linear Griffin-Lim restatement (fp64, scipy.fftpack, single-threaded) for ONE config-5
    sentence (sentence 0: its L, speaker 0, style mel 0), full 500-step cap and 60 GL iterations."""
    from oracle.griffin_lim_oracle import AudioOracle
    from oracle.tacotron_torch import TacotronTorchCPU
    cfg = gu.default_config("config_tacotron_gst.json")
    o = TacotronTorchCPU(weights.tacotron_gst_weights(0, num_speakers=4), r=cfg.r, memory_size=cfg.memory_size,
                         attn_norm=cfg.attention_norm, forward_attn=cfg.use_forward_attn,
                         trans_agent=cfg.transition_agent, forward_attn_mask=cfg.forward_attn_mask,
                         location_attn=cfg.location_attn, attn_win=cfg.windowing, max_decoder_steps=500)
    ap = AudioOracle(**{**cfg.audio, "griffin_lim_iters": args.iters})
    L = int(weights.synthetic_lengths(1, 4)[0])
    ids = weights.synthetic_ids(L, 200)
    style = np.random.Generator(np.random.PCG64(4)).uniform(0, 1, size=(1, 200, 80)).astype(np.float32)[0]
    threads, how = _physical_cores()
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        o.inference(ids[:8], 0, style)  # warm (allocator, thread pool)
        t0 = time.time()
        res = o.inference(ids, 0, style)
        t_model = time.time() - t0
        np.random.seed(0)
        ap.inv_spectrogram(res["linear"].T)
        dt = time.time() - t0
    finally:
        torch.set_num_threads(prev_threads)
    T = res["mel"].shape[0]
    return dict(value=T / dt, unit="mel-frames/s", cores=int(threads), cores_how=how, kind="port",
                cpu_model=_cpu_model(),
                sample=f"1 config-5 sentence (L={L}, {T} frames): torch-CPU TacotronGST (fp32, {threads} threads, "
                       f"{t_model:.2f} s) + linear GL {args.iters} iters (fp64, scipy.fftpack, single-threaded) on the "
                       f"host, {dt:.1f} s",
                model_half_frames_per_s=T / t_model, port_over_reference=_port_over_reference("gst_model"),
                rtf=dt / (275 * (T - 1) / 22050.0))


def cpu_baseline(args, seconds_target=12.0):
    """The reference's CPU path restated on the host: torch-CPU decoder + postnet
    (oracle/tacotron2_torch.py, the reference's op order on the same torch CPU kernels) on the
    process's physical cores + the numpy Griffin-Lim restatement (fp64, scipy.fftpack,
    single-threaded like librosa's)."""
    from oracle.griffin_lim_oracle import AudioOracle
    from oracle.tacotron2_torch import Tacotron2TorchCPU
    if args.model == "gst":
        return cpu_baseline_gst(args)
    threads, how = _physical_cores()
    cfg = gu.default_config("config_tacotron2.json")
    o = Tacotron2TorchCPU(weights.tacotron2_weights(0), attn_norm=cfg.attention_norm,
                          forward_attn=cfg.use_forward_attn, trans_agent=cfg.transition_agent,
                          forward_attn_mask=True, location_attn=cfg.location_attn, attn_win=cfg.windowing)
    ap = AudioOracle(**{**cfg.audio, "griffin_lim_iters": args.iters})
    ids = weights.synthetic_ids(args.L, 1)
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        o.inference(ids)  # warm (allocator, BLAS thread pool)
        frames = 0
        n = 0
        t_model = 0.0
        t0 = time.time()
        while True:
            tm = time.time()
            res = o.inference(ids)
            t_model += time.time() - tm
            np.random.seed(n)
            ap.inv_mel_spectrogram(res["mel_post"].T)
            frames += res["mel"].shape[0]
            n += 1
            if time.time() - t0 >= seconds_target or n >= 8:
                break
        dt = time.time() - t0
        # configs[0]: the reference's own CPU case, synthesize.py with 30-iteration Griffin-Lim, one sentence
        ap30 = AudioOracle(**{**cfg.audio, "griffin_lim_iters": 30})
        t1 = time.time()
        r30 = o.inference(ids)
        np.random.seed(0)
        ap30.inv_mel_spectrogram(r30["mel_post"].T)
        d30 = time.time() - t1
    finally:
        torch.set_num_threads(prev_threads)
    T30 = r30["mel"].shape[0]
    T = res["mel"].shape[0]
    return dict(value=frames / dt, unit="mel-frames/s", cores=int(threads), kind="port",
                cores_how=how,
                sample=f"{n} x one L={args.L} sentence ({T} frames): torch-CPU restatement decoder+postnet "
                       f"(fp32, {threads} threads, {t_model / n:.3f} s/sentence) + GL {args.iters} iters (fp64, "
                       f"scipy.fftpack, single-threaded) on the host, {dt:.1f} s",
                model_half_frames_per_s=frames / t_model,
                port_over_reference=_port_over_reference(),
                rtf=dt / (n * 275 * (T - 1) / 22050.0), cpu_model=_cpu_model(),
                configs0=dict(value=T30 / d30, unit="mel-frames/s", seconds=d30, rtf=d30 / (275 * (T30 - 1) / 22050.0),
                              sample=f"configs[0]: one L={args.L} sentence ({T30} frames), GL 30 iters, same port"))


def load_traffic(kernel):
    """HBM bytes per launch from the committed PMC summary (profiles/pmc_*.json), or None."""
    for p in sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_*.json")), reverse=True):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if kernel in d.get("per_launch_hbm_bytes", {}):
            return d["per_launch_hbm_bytes"][kernel]
    return None


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def timed_region(step, args, world, device, hop, sr):
    """W untimed warmup steps, then EXACTLY K timed steps bracketed by barrier + device sync on both
    sides; the MAX elapsed over ranks, the SUM of frames / audio seconds over ranks (driver contract).
    ``step(seed)`` runs one step and returns this rank's per-sentence frame counts."""
    for w in range(args.warmup):
        step(w)
    _sync(device)
    if world > 1:
        dist.barrier()
    _sync(device)
    t0 = time.perf_counter()
    frames = []
    for k in range(args.steps):
        frames = step(1000 + k)
    _sync(device)
    if world > 1:
        dist.barrier()
    _sync(device)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    nfr = torch.tensor([float(sum(frames))], dtype=torch.float64, device=device)
    aud = torch.tensor([sum(hop * (f - 1) for f in frames) / sr], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(nfr)
        dist.all_reduce(aud)
    elapsed = float(t.item())
    frames_per_step = float(nfr.item())
    return dict(elapsed=elapsed, frames_per_step=frames_per_step, ms_per_step=1000.0 * elapsed / args.steps,
                value=frames_per_step * args.steps / elapsed, rtf=(elapsed / args.steps) / float(aud.item()))


def proxy_main(args, world, rank):
    """CPU rehearsal of the multi-rank bench (``--backend gloo --proxy``): the same launcher, rank
    environment, configs[3] job + LPT share, timed region and gather-v of finished waveforms, with
    each sentence's waveform replaced by a deterministic stand-in of its length.  Tests the plumbing
    only: the line it prints carries ``"proxy": true`` and is not a measurement."""
    if world > 1:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus
    cpu = torch.device("cpu")
    all_ids, mine = make_job(args, world, rank, 1000)
    hop = 275

    def make_step(ids, share, w):
        def step(seed):
            frames = [sharding.sentence_cost(len(ids[i]), 1000) for i in share]
            rows = [torch.from_numpy(np.random.Generator(np.random.PCG64(i)).standard_normal(hop * (T - 1)))
                    for i, T in zip(share, frames)]
            if w > 1:
                sharding.gather_waveforms(rows, share, len(ids))
            return frames
        return step

    ref = single_rank_reference(make_step(all_ids, mine, 1), args, world, rank, cpu, hop, 22050)
    tm = timed_region(make_step(all_ids, mine, world), args, world, cpu, hop, 22050)
    share = None
    if world == 1 and args.model != "gst":
        ids8, mine8 = configs3_share(args, 1000)
        share = share_record(timed_region(make_step(ids8, mine8, 1), args, 1, cpu, hop, 22050), len(mine8))
    if rank == 0:
        rec = {"metric": "proxy (launcher rehearsal, not a measurement)", "value": tm["value"],
               "unit": "mel-frames/s", "n_gpus": world,
               "world_size_seen": dist.get_world_size() if world > 1 else 1, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": tm["ms_per_step"], "proxy": True,
               "config": {"sentences_per_gpu": args.batch, "sentences_total": len(all_ids),
                          "frames_per_step": tm["frames_per_step"], "lengths": args.lengths}}
        rec.update(scaling_keys(tm, ref, world, share))
        print(json.dumps(rec))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def single_rank_reference(step, args, world, rank, device, hop, sr):
    """N > 1: rank 0 times its own share ALONE (the same synthesis, no gather) while every other rank
    waits at a barrier, before the collective timed region: the single-GPU point of this very
    per-rank workload, so the line carries its own weak-scaling reference.  None at N = 1 or on
    ranks > 0."""
    if world == 1:
        return None
    dist.barrier()
    ref = None
    if rank == 0:
        ref = timed_region(step, args, 1, device, hop, sr)
    dist.barrier()
    return ref


def share_record(tm, n_sentences=None):
    d = dict(value=tm["value"], unit="mel-frames/s", ms_per_step=tm["ms_per_step"],
             frames_per_step=tm["frames_per_step"], rtf=tm["rtf"])
    if n_sentences is not None:
        d["sentences"] = n_sentences
    return d


def scaling_keys(tm, ref, world, share):
    """Keys that make the 1/2/4/8-GPU records comparable: at N > 1
    ``scaling_ref_1rank`` (rank 0's share timed alone on one GPU) and ``efficiency`` =
    value / (N x scaling_ref_1rank); at N = 1 ``configs3_share_1rank`` (rank 0's share of the
    8-GPU configs[3] job on this one GPU), beside the configs[1] headline."""
    out = {}
    if ref is not None:
        r = share_record(ref)
        r["note"] = "rank 0's share of this job, timed alone on one GPU before the collective region (no gather)"
        out["scaling_ref_1rank"] = r
        out["efficiency"] = tm["value"] / (world * ref["value"])
    if share is not None:
        share["note"] = ("rank 0's LPT share of configs[3] (512 seed-3 sentences over 8 GPUs) on this one GPU: "
                         "the per-rank workload of the N=8 line")
        out["configs3_share_1rank"] = share
    return out


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(nproc, argv):
    """``--gpus N`` without a launcher around us: start torch.distributed.run with N ranks on this
    node as a CHILD process (nothing here has touched the GPU yet) and return its exit code; every
    rank re-enters this script with RANK / LOCAL_RANK / WORLD_SIZE set (reference process-per-GPU
    launcher: distribute.py:129-167)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def parse_args(argv=None):
    ap_ = argparse.ArgumentParser()
    ap_.add_argument("--gpus", type=int, default=1)
    ap_.add_argument("--steps", type=int, default=10)
    ap_.add_argument("--warmup", type=int, default=3)
    ap_.add_argument("--batch", type=int, default=None,
                     help="sentences per rank (default: 1 = configs[1] at N=1, 64 = configs[3] at N>1)")
    ap_.add_argument("--L", type=int, default=100)
    ap_.add_argument("--lengths", choices=["fixed", "uniform"], default=None,
                     help="fixed L (configs[1]) or L ~ U{60..160} (configs[2]/[3]); default by N")
    ap_.add_argument("--iters", type=int, default=60)
    ap_.add_argument("--no-cpu-baseline", action="store_true")
    ap_.add_argument("--no-profile", action="store_true")
    ap_.add_argument("--no-share", action="store_true",
                     help="N=1: skip the configs[3]-share region (configs3_share_1rank)")
    ap_.add_argument("--model", choices=["tacotron2", "gst"], default="tacotron2")
    ap_.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                     help="gloo + --proxy: CPU rehearsal of the launcher / partition / gather (no GPU)")
    ap_.add_argument("--proxy", action="store_true",
                     help="replace the GPU synthesis by a deterministic stand-in waveform per sentence "
                          "(launcher test only: the printed value is not a measurement)")
    args = ap_.parse_args(argv)
    if args.batch is None:
        args.batch = 32 if args.model == "gst" else (64 if args.gpus > 1 else 1)
    if args.lengths is None:
        args.lengths = "uniform" if args.batch > 1 else "fixed"
    return args


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if args.proxy:
        return proxy_main(args, world, rank)
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group(args.backend, device_id=device if args.backend == "nccl" else None)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)

    cfg, model, ap = build(args, device)
    all_ids, mine = make_job(args, world, rank, model.decoder.max_decoder_steps)
    ids = [all_ids[i] for i in mine]

    # N > 1: rank 0's share alone first (same synthesis, no gather; the other ranks wait)
    ref = single_rank_reference(lambda seed: run_step(model, ap, all_ids, mine, 1, seed=seed)[0], args, world, rank,
                                device, ap.hop_length, ap.sample_rate)
    if ref is not None:
        collect_status(model)
    timing = timed_region(lambda seed: run_step(model, ap, all_ids, mine, world, seed=seed)[0], args, world, device,
                          ap.hop_length, ap.sample_rate)
    collect_status(model)
    elapsed, frames_per_step, ms_per_step, value, rtf = (timing[k] for k in ("elapsed", "frames_per_step",
                                                                           "ms_per_step", "value", "rtf"))

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    # ---- per-stage wall times (rank 0, one extra untimed step) and per-kernel profile
    gst = args.model == "gst"
    if not gst:  # the timed loop ran tts_synth_run: warm the per-stage entry points (graphs, buffers) once
        warm = model.inference_batch(ids)
        ap.griffin_lim_batch(warm["mel_post"], warm["frames"], seed=7)
    torch.cuda.synchronize()
    s0 = time.perf_counter()
    if gst:
        style, spk = gst_inputs(len(all_ids), device)
        sel = torch.as_tensor(mine, dtype=torch.long, device=device)
        out = model.inference_batch(ids, speaker_ids=[spk[i] for i in mine], style_mel=style.index_select(0, sel))
    else:
        out = model.inference_batch(ids)
    torch.cuda.synchronize()
    s1 = time.perf_counter()
    if gst:
        ap.griffin_lim_batch(out["linear"], out["frames"], mode=audiomod._native.TTS_GL_FROM_LINEAR, seed=7)
    else:
        ap.griffin_lim_batch(out["mel_post"], out["frames"], seed=7)
    torch.cuda.synchronize()
    s2 = time.perf_counter()
    dec_ms = model.last_timing.get("decoder_loop_ms", 0.0)
    gl_ms = ap.last_gl_timing()["gl_loop_ms"]
    stages = dict(tacotron2_ms=1000 * (s1 - s0), decoder_loop_ms=dec_ms, griffin_lim_ms=1000 * (s2 - s1),
                  gl_iteration_loop_ms=gl_ms)
    roofline = None
    kernels = {}
    if not args.no_profile:
        B = len(ids)
        Lmean = float(np.mean([len(x) for x in ids]))
        steps = max(out["steps"])
        frames_total = sum(out["frames"])
        resident = bool(model.last_timing.get("resident", False))
        # resident decoders: ONE launch runs every step (csrc/resident_decoder.hip for the batch-1
        # Tacotron2, csrc/tacotron_resident.hip for the TacotronGST batch), timed with HIP events on
        # the library stream around that launch; otherwise the per-step kernels
        kd = {} if resident else model.profile_step_kernels(reps=50 if not gst else 20)
        # small batches run every GL iteration after the first in ONE persistent launch
        # (griffin_lim.hip: gl_persistent_kernel), timed with HIP events around it
        gl_persistent = ap.last_gl_timing()["gl_iterations"] == 1 and args.iters > 1
        kg = {} if gl_persistent else ap.profile_gl_kernels(reps=20)
        launches = {k: steps for k in kd}
        allk = dict(kd)
        if not gl_persistent:
            # one GL iteration = overlap-add launch (frames -> float32 signal) + per-frame
            # STFT/iSTFT launch; priced together against SURVEY 8(d)'s bytes per frame-iteration
            launches["gl_iter"] = args.iters
            allk["gl_iter"] = kg["gl_iter"] + kg["gl_ola"]
        for k, ms in allk.items():
            kind, alg = (kernel_algorithmic_gst if gst else kernel_algorithmic)(k, B, Lmean, frames_total)
            kernels[k] = dict(mean_ms=ms, launches_per_step=launches[k], ms_per_step=ms * launches[k],
                              algorithmic_bytes=alg, achieved_gbs=alg / (ms * 1e-3) / 1e9 if ms > 0 else None)
        if resident and gst:
            # the per-step kernels' algorithmic bytes (weights once per batch-step) x steps
            alg = sum(kernel_algorithmic_gst(k, B, Lmean, frames_total)[1]
                      for k in audiomod._native.TACOTRON_STEP_KERNELS) * steps
            kernels["tacotron_resident"] = dict(mean_ms=dec_ms, launches_per_step=1, ms_per_step=dec_ms,
                                                decoder_steps=steps, us_per_decoder_step=1000 * dec_ms / steps,
                                                algorithmic_bytes=alg, achieved_gbs=alg / (dec_ms * 1e-3) / 1e9)
        elif resident:
            alg = decoder_step_algorithmic(B, Lmean) * steps
            kernels["resident_decoder"] = dict(mean_ms=dec_ms, launches_per_step=1, ms_per_step=dec_ms,
                                               decoder_steps=steps, us_per_decoder_step=1000 * dec_ms / steps,
                                               algorithmic_bytes=alg, achieved_gbs=alg / (dec_ms * 1e-3) / 1e9,
                                               phases_us_per_step=model.profile_resident_phases())
        if gl_persistent:
            alg = GL_BYTES_PER_FRAME_ITER * frames_total * args.iters
            kernels["gl_persistent"] = dict(mean_ms=gl_ms, launches_per_step=1, ms_per_step=gl_ms,
                                            gl_iterations=args.iters, us_per_iteration=1000 * gl_ms / args.iters,
                                            algorithmic_bytes=alg, achieved_gbs=alg / (gl_ms * 1e-3) / 1e9)
        dom = max(kernels, key=lambda k: kernels[k]["ms_per_step"])
        kdom = kernels[dom]
        traffic = load_traffic(("gst_" if gst else "") + dom)
        roofline = dict(bound="hbm", kernel=dom, achieved=kdom["achieved_gbs"], peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=kdom["achieved_gbs"] / HBM_PEAK_GBS, traffic=traffic,
                        algorithmic_bytes_per_launch=kdom["algorithmic_bytes"], mean_launch_ms=kdom["mean_ms"])
        hbm_equivalent = dict(roofline)
        if traffic:
            roofline["traffic_over_algorithmic"] = traffic / kdom["algorithmic_bytes"]
        if dom in ("gl_iter", "gl_persistent"):
            # the fp64 STFT/iSTFT of every frame: the SURVEY 8(d) byte count prices the |S| read and
            # the float32 signal, but the kernel's time goes to fp64 FFT passes through LDS
            flops = GL_FLOPS_PER_FRAME_ITER * frames_total * (1 if dom == "gl_iter" else args.iters)
            tf = flops / (kdom["mean_ms"] * 1e-3) / 1e12
            roofline["diagnostics"] = dict(
                limiter="batched: one wave per frame (gl_iter_wave_kernel), fp64 VALU (~65% busy) and the "
                        "vector-memory return path (TD ~74% busy); HBM traffic beyond the algorithmic bytes "
                        "is the float32 windowed frames written by the iteration launch and read back by the "
                        "overlap-add launch. Batch 1 (persistent loop): per iteration ~1.8 us of neighbour "
                        "hand-off (tagged float32 granules, two ping-pong slots) and ~4 us of fp64 FFT + "
                        "spectrum on one wave per SIMD (latency-bound LDS passes)",
                fp64_flops_per_launch=flops, fp64_tflops=tf, fp64_vector_frac=tf / FP64_VECTOR_PEAK_TF,
                traffic_gbs=(traffic / (kdom["mean_ms"] * 1e-3) / 1e9) if traffic else None)
        if dom == "resident_decoder":
            # the SURVEY 8(d) HBM figure prices a weight stream the resident kernel never does (its
            # weights stay in VGPRs / LDS): state what actually bounds it
            flops = decoder_step_flops(Lmean) * steps
            ph = kdom["phases_us_per_step"]["cu0"]
            # round 4 made the prenet-1 edge XCD-local: two device-wide edges (h_att, h_dec: every
            # CU's LSTM rows need all of h) and four XCD-local ones (pre1, prenet-2, query, context)
            dev_edges = {k: ph[k] for k in ("att_cell_gather", "dec_cell_gather")}
            xcd_edges = {k: ph[k] for k in ("att_early_wait_pre1", "wait_prenet2", "wait_query", "wait_ctx")}
            us = kdom["us_per_decoder_step"]
            floor = 2 * EDGE_DEVICE_US + 4 * EDGE_XCD_US
            roofline["diagnostics"] = dict(
                limiter="hand-off latency: 2 device-wide + 4 XCD-local edges per step; weights on chip",
                fp32_flops_per_launch=flops, fp32_tflops=flops / (dec_ms * 1e-3) / 1e12,
                fp32_compute_frac=flops / (dec_ms * 1e-3) / 1e12 / FP32_MFMA_PEAK_TF,
                device_wide_edges_us_per_step=dev_edges, xcd_local_edges_us_per_step=xcd_edges,
                edge_microbench_us=dict(device_wide=EDGE_DEVICE_US, xcd_local=EDGE_XCD_US,
                                        source="tools/microbench/edge.hip (one 16-byte granule pair per lane, best first-poll delay; profiles/r06_edge_floor.log)"),
                latency_floor_us=floor, step_over_floor=us / floor, us_per_step=us)
            # the resident decoder's weights never leave the chip (counter traffic ~1 % of the SURVEY
            # 8(d) bytes): its roofline is the hand-off latency floor, not HBM.  The
            # HBM-equivalent figure stays as a labelled diagnostic.
            hbm_equivalent.pop("traffic", None)
            roofline.update(bound="latency", achieved=us, peak=floor, unit="us/decoder-step", frac=floor / us)
            roofline["diagnostics"]["hbm_equivalent"] = dict(
                hbm_equivalent, note="SURVEY 8(d) algorithmic bytes per step x steps / launch time: what a weight "
                                     "stream would have to sustain; the kernel reads its weights once per launch")
    # the headline workload's paths, before any other region runs on the same handles
    paths = dict(decoder="resident" if model.last_timing.get("resident") else "multi-launch",
                 encoder_bilstm={1: "resident", 2: "resident-batched"}.get(model.last_timing.get("encoder_path", 0), "per-step")
                 if not gst else "bigru_kernel (the CBHG / GST recurrences: one launch each; the only path)",
                 griffin_lim=ap.last_gl_path())
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)
    server = None
    if world == 1 and not gst and not args.no_share:
        # the Synthesizer.tts() configuration on the same L=100 sentence (mask off: it runs to the
        # 3000-step cap under random weights), one sentence per step through the same one-call path;
        # bounded to 3 timed steps (~35 ms each)
        sm = build_server_model(args)
        sargs = argparse.Namespace(**{**vars(args), "steps": min(args.steps, 3), "warmup": 1})
        tm = timed_region(lambda seed: run_step(sm, ap, ids, [0], 1, seed=seed)[0], sargs, 1, device, ap.hop_length,
                          ap.sample_rate)
        collect_status(sm)
        server = share_record(tm, 1)
        server.update(steps=sargs.steps, decoder="resident" if sm.last_timing.get("resident") else "multi-launch",
                      note="Synthesizer.tts()'s model (config_tacotron2.json: forward attention, sigmoid, mask off, "
                           "3000-step cap; server/synthesizer.py:46-66), one L=100 sentence per step, GL "
                           f"{args.iters} iters: the general-form resident decoder")
        del sm
    tts_wall = None
    if world == 1 and not gst and not args.no_share:
        tts_wall = synthesizer_tts_wall(args, ap, server["ms_per_step"] if server else None)
    share = None
    if world == 1 and not gst and not args.no_share:
        # the driver's N=8 line runs configs[3]'s 64-sentence share per rank: time that same share
        # here on one GPU (after the headline and its profile, which keep their batch-1 handles)
        ids8, mine8 = configs3_share(args, model.decoder.max_decoder_steps)
        share = share_record(timed_region(lambda seed: run_step(model, ap, ids8, mine8, 1, seed=seed)[0], args, 1,
                                          device, ap.hop_length, ap.sample_rate), len(mine8))
        collect_status(model)

    if gst:
        workload = (f"configs[4]: TacotronGST batch={args.batch} per GPU, L ~ U{{60..160}}, style mel [B,200,80], "
                    f"4 speakers, linear GL {args.iters} iters")
    elif args.batch == 1:
        workload = f"configs[1]: Tacotron2 single sentence, HIP decoder loop + HIP Griffin-Lim {args.iters} iters"
    elif world > 1 and args.lengths == "uniform":
        workload = (f"configs[3]: Tacotron2, {len(all_ids)} sentences (L ~ U{{60..160}}, seed 3) LPT-sharded "
                    f"{args.batch} per GPU over {world} GPUs, GL {args.iters} iters, RCCL gather-v to rank 0")
    elif args.batch == 64 and args.lengths == "uniform":
        workload = f"configs[2]: Tacotron2 batch=64, L ~ U{{60..160}} (seed 2), GL {args.iters} iters"
    else:
        workload = f"Tacotron2 batch={args.batch} per GPU, {args.lengths} lengths"
    rec = {
        "metric": ("mel-frames/sec + RTF, TacotronGST + 60-iter Griffin-Lim (configs[4])" if gst else
                   "mel-frames/sec + RTF, Tacotron2 + 60-iter Griffin-Lim, LJSpeech"),
        "value": value,
        "unit": "mel-frames/s",
        "n_gpus": world,
        "world_size_seen": dist.get_world_size() if world > 1 else 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic ids, random-init weights (deterministic generator, seed 0)",
        "config": {"workload": workload,
                   "sentences_per_gpu": args.batch,
                   "L": args.L if (args.lengths == "fixed" and not gst) else "U{60..160}",
                   "frames_per_step": frames_per_step, "gl_iters": args.iters,
                   "model_config": ("config_tacotron_gst.json, num_speakers=4" if gst else
                                    "config_tacotron2.json + forward_attn_mask (synthesize.py:86)"),
                   "parallelism": (f"sentence-sharded x{world} (LPT), RCCL gather-v of waveforms to rank 0"
                                   if world > 1 else "single GPU")},
        "rtf": rtf,
        "roofline": roofline,
        "cpu_baseline": cpu,
        "stages_rank0": stages,
        "paths_rank0": paths,
        "kernels_rank0": kernels,
    }
    rec.update(scaling_keys(timing, ref, world, share))
    if server is not None:
        rec["synthesizer_config_1rank"] = server
    if tts_wall is not None:
        rec["synthesizer_tts_wall"] = tts_wall
    print(json.dumps(rec))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
