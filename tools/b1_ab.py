"""A/B helper (GPU box): configs[1] ids -> wav wall time per sentence (tts_synth_run, pipelined as the
bench runs it) for the library named by TTS_HIP_LIB (measurement only)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import load_pkg, weights_mod  # noqa: E402

gu = load_pkg("generic_utils")
audio = load_pkg("audio")
cfg = gu.default_config("config_tacotron2.json")
cfg.forward_attn_mask = True
m = gu.setup_model(130, cfg, max_batch=1, max_len=256).cuda().eval()
ap = audio.AudioProcessor(**cfg.audio)
ids = weights_mod().synthetic_ids(100, 1)
for k in range(5):
    m.synthesize_native([ids], ap, seed=k, sync=False)
m.synth_sync()
reps = []
for r in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(20):
        m.synthesize_native([ids], ap, seed=k, sync=False)
    torch.cuda.synchronize()
    reps.append((time.perf_counter() - t0) / 20 * 1e3)
m.synth_sync()
print(json.dumps(dict(ms_per_sentence=float(np.median(reps)), min=float(min(reps)), max=float(max(reps)),
                      gl_path=ap.last_gl_path(), decoder_ms=m.last_timing["decoder_loop_ms"])))
