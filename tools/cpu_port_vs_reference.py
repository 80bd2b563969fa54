"""the CPU port (oracle/) timed against the REFERENCE on the same cores.

Build container only (imports /root/reference; nothing here runs on the GPU box):

    python tools/cpu_port_vs_reference.py [out.json]

configs[1]'s model half: one L=100 sentence (ids seed 1, generator weights seed 0,
config_tacotron2.json + forward_attn_mask) through the reference ``Tacotron2.inference`` (imported
with the text front-end stubbed, as tests/golden/make_golden.py does) and through the oracle's
torch-CPU restatement ``Tacotron2TorchCPU.inference`` (bench.py's cpu_baseline model half), plus the
numpy ``Tacotron2Oracle.inference`` (float32) for the record, at 8 threads and at 1 thread
(torch.set_num_threads, and threadpoolctl's BLAS limit for numpy).  Griffin-Lim half: the reference
``AudioProcessor.inv_mel_spectrogram`` with librosa replaced by the oracle's restatement (librosa
is absent here) against ``AudioOracle.inv_mel_spectrogram``, 60 iterations, on the reference's own
mel_post, same initial phases.  Medians of several runs; the ratio port / reference is what
section 3.2 asks to be within 10 %.
"""
import json
import os
import statistics
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
sys.path.insert(0, REPO)

import make_golden as mg  # noqa: E402  (stubs + weights loader; generates nothing on import)
from conftest import golden, golden_flags, tacotron2_config  # noqa: E402
from oracle.griffin_lim_oracle import AudioOracle  # noqa: E402
from oracle.tacotron2_oracle import Tacotron2Oracle  # noqa: E402
from oracle.tacotron2_torch import Tacotron2TorchCPU  # noqa: E402


def median_time(fn, reps):
    fn()  # warm
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts), ts


def main(out_path):
    import torch
    from threadpoolctl import threadpool_limits

    mg._stub_text_deps()
    mg._stub_audio_deps()
    sys.path.insert(0, mg.REF)
    from utils.audio import AudioProcessor
    from utils.generic_utils import load_config, setup_model

    C = load_config(os.path.join(mg.REF, "config_tacotron2.json"))
    C.num_speakers = 0
    C.forward_attn_mask = True
    model = setup_model(130, 0, C)
    sd = mg.weights.tacotron2_weights(0, num_chars=130)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model.eval()
    ids = mg.weights.synthetic_ids(100, 1)
    x = torch.from_numpy(ids).unsqueeze(0)
    fl = golden_flags(golden("t2_fwdmask_L100"))
    port = Tacotron2TorchCPU(sd, **fl)
    port_np = Tacotron2Oracle(sd, dtype=np.float32, **fl)

    res = {"workload": "configs[1] model half: Tacotron2 inference, one L=100 sentence (222 frames)",
           "cpu_model": _cpu_model(), "model": {}, "griffin_lim": {}}
    mel_post = None
    for threads in (8, 4, 1):
        torch.set_num_threads(threads)

        def ref_run():
            with torch.no_grad():
                return model.inference(x)

        with threadpool_limits(limits=threads, user_api="blas"):
            # interleaved medians (this host's 8 threads are noisy): reference, port, reference, port
            trs, tps = [], []
            for _ in range(2):
                trs += median_time(ref_run, 4 if threads > 1 else 2)[1]
                tps += median_time(lambda: port.inference(ids), 4 if threads > 1 else 2)[1]
            tr, tp = statistics.median(trs), statistics.median(tps)
            tn, _ = median_time(lambda: port_np.inference(ids), 3)
        if mel_post is None:
            mel_post = ref_run()[1][0].numpy()
        res["model"][f"threads_{threads}"] = dict(reference_s=tr, port_s=tp, port_over_reference=tp / tr,
                                                  numpy_oracle_s=tn, numpy_over_reference=tn / tr)
        print(threads, "threads: reference", tr, "torch port", tp, "ratio", tp / tr, "numpy", tn, flush=True)

    # configs[4]'s model half: the reference TacotronGST (config_tacotron_gst.json, 4 speakers) on
    # config-5 sentence 0 (its L, speaker 0, style mel 0, 500-step cap) vs oracle/tacotron_torch.py
    from oracle.tacotron_torch import TacotronTorchCPU
    Cg = load_config(os.path.join(mg.REF, "config_tacotron_gst.json"))
    Cg.num_speakers = 4
    gmodel = setup_model(130, 4, Cg)
    gsd = mg.weights.tacotron_gst_weights(0, num_speakers=4)
    gmodel.load_state_dict({k: torch.from_numpy(v) for k, v in gsd.items()})
    gmodel.eval()
    gport = TacotronTorchCPU(gsd, r=Cg.r, memory_size=Cg.memory_size, attn_norm=Cg.attention_norm,
                             forward_attn=Cg.use_forward_attn, trans_agent=Cg.transition_agent,
                             forward_attn_mask=Cg.forward_attn_mask, location_attn=Cg.location_attn,
                             attn_win=Cg.windowing, max_decoder_steps=500)
    Lg = int(mg.weights.synthetic_lengths(1, 4)[0])
    gids = mg.weights.synthetic_ids(Lg, 200)
    style = np.random.Generator(np.random.PCG64(4)).uniform(0, 1, size=(1, 200, 80)).astype(np.float32)
    gx, gstyle, gspk = torch.from_numpy(gids)[None], torch.from_numpy(style), torch.tensor([0])
    res["gst_workload"] = f"configs[4] model half: TacotronGST inference, one L={Lg} sentence, 500-step cap"
    res["gst_model"] = {}
    for threads in (8, 4, 1):
        torch.set_num_threads(threads)

        def gref():
            with torch.no_grad():
                return gmodel.inference(gx, speaker_ids=gspk, style_mel=gstyle)

        trs, tps = [], []
        for _ in range(2):
            trs += median_time(gref, 2 if threads > 1 else 1)[1]
            tps += median_time(lambda: gport.inference(gids, 0, style[0]), 2 if threads > 1 else 1)[1]
        tr, tp = statistics.median(trs), statistics.median(tps)
        res["gst_model"][f"threads_{threads}"] = dict(reference_s=tr, port_s=tp, port_over_reference=tp / tr)
        print("GST", threads, "threads: reference", tr, "torch port", tp, "ratio", tp / tr, flush=True)

    # Griffin-Lim 60: reference AudioProcessor glue (librosa = the restatement) vs AudioOracle
    a = dict(tacotron2_config()["audio"])
    a["griffin_lim_iters"] = 60
    ref_ap = AudioProcessor(**{k: v for k, v in a.items() if k in AudioProcessor.__init__.__code__.co_varnames})
    port_ap = AudioOracle(**a)

    def ref_gl():
        np.random.seed(0)
        return ref_ap.inv_mel_spectrogram(mel_post.T)

    def port_gl():
        np.random.seed(0)
        return port_ap.inv_mel_spectrogram(mel_post.T)

    with threadpool_limits(limits=1, user_api="blas"):
        tr, _ = median_time(ref_gl, 3)
        tp, _ = median_time(port_gl, 3)
    res["griffin_lim"] = dict(iters=60, frames=int(mel_post.shape[0]), reference_s=tr, port_s=tp,
                              port_over_reference=tp / tr,
                              note="librosa is absent: the reference glue runs over the oracle's librosa-0.6.2 "
                                   "restatement, so this compares the glue, not librosa's own FFT code")
    print("GL 60: reference", tr, "port", tp, "ratio", tp / tr)
    json.dump(res, open(out_path, "w"), indent=1)
    print("wrote", out_path)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip() + f" ({os.cpu_count()} logical CPUs visible)"
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "profiles", "cpu_port_vs_reference_r05.json"))
