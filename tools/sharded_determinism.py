"""Measurement (GPU box): is synthesize_batch deterministic across calls, and which decode path does
each call of tests/test_gpu_parity.py::test_sharded_synthesis_single_rank take?  Prints per call
the dispatch, the per-sentence resident flags and the max |diff| of mel_post / waveform vs call 0."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import golden, golden_flags, load_pkg, weights_mod  # noqa: E402

t2 = load_pkg("tacotron2")
synth = load_pkg("synthesis")
audio = load_pkg("audio")
cfg = load_pkg("generic_utils").default_config("config_tacotron2.json")
fl = golden_flags(golden("t2_fwdmask_L12"))
m = t2.Tacotron2(130, 0, r=1, attn_win=fl["attn_win"], attn_norm=fl["attn_norm"], forward_attn=fl["forward_attn"],
                 trans_agent=fl["trans_agent"], forward_attn_mask=fl["forward_attn_mask"],
                 location_attn=fl["location_attn"])
m.decoder.max_decoder_steps = fl["max_decoder_steps"]
m = m.cuda().eval()
ap = audio.AudioProcessor(**{**cfg.audio, "griffin_lim_iters": 5})
w = weights_mod()
ids = [w.synthetic_ids(L, 7 + L) for L in (9, 17, 4)]
ref = None
for call in range(4):
    wavs, info = synth.synthesize_batch(m, ap, ids, seed=11, phase="device", keep_outputs=(call % 2 == 0))
    mp = info["mel_post"].float().cpu().numpy() if "mel_post" in info else None
    wv = [np.asarray(x.cpu().numpy() if torch.is_tensor(x) else x) for x in wavs]
    if ref is None:
        ref = (mp, wv)
    dm = None if mp is None or ref[0] is None else float(np.abs(mp - ref[0]).max())
    dw = max(float(np.abs(a - b).max()) for a, b in zip(wv, ref[1]))
    print(call, info.get("decoder_dispatch"), m.last_timing.get("resident"), "mel_post maxdiff", dm, "wav maxdiff", dw,
          flush=True)
