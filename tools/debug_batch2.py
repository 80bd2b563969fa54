"""Debug helper (GPU): which sentences of a batch differ from their batch-1 run (mel, encoder)."""
import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
w = importlib.import_module("your-voice-tts_amd.weights")
t2 = importlib.import_module("your-voice-tts_amd.tacotron2")
fl = dict(attn_norm="sigmoid", forward_attn=True, trans_agent=False, forward_attn_mask=True, location_attn=False)
m = t2.Tacotron2(130, 0, r=1, **fl)
m.load_state_dict({k: torch.from_numpy(v) for k, v in w.tacotron2_weights(0).items()})
m.cuda().eval()
lens = w.synthetic_lengths(64, 2)
ids = [w.synthetic_ids(int(L), 100 + b) for b, L in enumerate(lens)]
for B in (40,):
    outB = m.inference_batch(ids[:B])
    lb = [len(x) for x in ids[:B]]
    pad = torch.zeros(B, max(lb), dtype=torch.long)
    for b, x in enumerate(ids[:B]):
        pad[b, :len(x)] = torch.from_numpy(np.asarray(x))
    encB = m.encode(pad.cuda(), lb)
    bad = []
    for b in range(B):
        one = m.inference_batch([ids[b]])
        T = one["frames"][0]
        d = (outB["mel"][b, :T] - one["mel"][0, :T]).abs().max().item()
        e1 = m.encode(pad[b:b + 1, :lb[b]].cuda(), [lb[b]])
        de = (encB[b, :lb[b]] - e1[0]).abs().max().item()
        if d > 1e-5 or de > 1e-5:
            bad.append((b, round(d, 6), round(de, 6)))
    print(f"B={B}: sentences differing from batch-1 (b, mel, enc): {bad}", flush=True)
