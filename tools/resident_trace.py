#!/usr/bin/env python3
"""Per-CU event trace of the resident batch-1 decoder at configs[1] (measurement only).

Re-runs the last sentence with timers (tts_decoder_resident_phases) and reads the event trace:
for each event, its spread across the 256 CUs relative to the step's first P1, and which CUs
are last to publish h_att / h_dec.

    python tools/resident_trace.py [--L 100]
"""
import argparse
import collections
import importlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
gu = importlib.import_module("your-voice-tts_amd.generic_utils")
weights = importlib.import_module("your-voice-tts_amd.weights")

EV = ("P1", "B1", "hatt_pub", "B3", "B4", "hdec_pub", "B6", "pre1_pub", "q_pub", "att_A1", "att_A2", "att_ctx_pub")

ap = argparse.ArgumentParser()
ap.add_argument("--L", type=int, default=100)
ap.add_argument("--nomask", action="store_true", help="Synthesizer.tts()'s configuration (general form)")
args = ap.parse_args()
cfg = gu.default_config("config_tacotron2.json")
cfg.forward_attn_mask = not args.nomask
m = gu.setup_model(130, cfg, max_batch=1, max_len=256)
m.load_state_dict({k: torch.from_numpy(v) for k, v in weights.tacotron2_weights(0).items()})
m.cuda().eval()
ids = weights.synthetic_ids(args.L, 1)
for _ in range(3):
    out = m.inference_batch([ids])
torch.cuda.synchronize()
ph = m.profile_resident_phases()
tr = m.profile_resident_trace().astype(np.float64) / 100.0  # wall clock 100 MHz -> us
steps = range(8, 60)
rel = {k: [] for k in EV}
last = {"hatt_pub": collections.Counter(), "hdec_pub": collections.Counter(), "pre1_pub": collections.Counter()}
period = []
for t in steps:
    t0 = tr[:, t, 0].min()
    period.append(tr[:, t + 1, 0].min() - t0)
    for k, name in enumerate(EV):
        v = tr[:, t, k]
        v = v[v > 0]
        if v.size == 0:  # (an event this form does not record)
            continue
        r = v - t0
        rel[name].append((r.min(), np.median(r), r.max()))
        if name in last:
            last[name][int(np.argmax(tr[:, t, k]))] += 1
rec = {"us_per_step_trace": float(np.median(period)),
       "events_rel_step_start_us(min,median,max)": {k: [round(float(x), 2) for x in np.median(np.array(v), 0)]
                                                    for k, v in rel.items() if v},
       "last_cu": {k: v.most_common(6) for k, v in last.items()},
       "phases": ph}
print(json.dumps(rec, indent=1))
