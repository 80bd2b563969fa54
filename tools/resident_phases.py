#!/usr/bin/env python3
"""Per-phase timing of the resident batch-1 decoder at configs[1] (measurement only).

    python tools/resident_phases.py [--L 100]
"""
import argparse
import importlib
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
gu = importlib.import_module("your-voice-tts_amd.generic_utils")
weights = importlib.import_module("your-voice-tts_amd.weights")

ap = argparse.ArgumentParser()
ap.add_argument("--L", type=int, default=100)
args = ap.parse_args()
cfg = gu.default_config("config_tacotron2.json")
cfg.forward_attn_mask = True
m = gu.setup_model(130, cfg, max_batch=1, max_len=256)
m.load_state_dict({k: torch.from_numpy(v) for k, v in weights.tacotron2_weights(0).items()})
m.cuda().eval()
ids = weights.synthetic_ids(args.L, 1)
for _ in range(3):
    out = m.inference_batch([ids])
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    out = m.inference_batch([ids])
torch.cuda.synchronize()
ph = m.profile_resident_phases()
steps = out["steps"][0]
rec = dict(L=args.L, steps=steps, resident=m.last_timing["resident"], decoder_loop_ms=m.last_timing["decoder_loop_ms"],
           us_per_step=1000 * m.last_timing["decoder_loop_ms"] / steps, phases=ph)
print(json.dumps(rec, indent=1))
