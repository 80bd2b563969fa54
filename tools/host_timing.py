"""Host-side timing of pipelined configs[1] tts_synth_run calls (measurement only): median call
duration and host time between calls; with 'sync' each call also waits for its Griffin-Lim."""
import os
import statistics
import sys
import time

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
ts = []
for k in range(40):
    a = time.perf_counter()
    m.synthesize_native([ids], ap, seed=k, sync=False)
    b = time.perf_counter()
    ts.append((a, b))
m.synth_sync()
dur = [(b - a) * 1e6 for a, b in ts]
gap = [(ts[i + 1][0] - ts[i][1]) * 1e6 for i in range(len(ts) - 1)]
per = [(ts[i + 1][0] - ts[i][0]) * 1e6 for i in range(len(ts) - 1)]
print("call us median %.1f  between calls %.1f  period %.1f" % (statistics.median(dur), statistics.median(gap),
                                                               statistics.median(per)))
