"""Measurement only: batch-1 decoder step kernels for the reference's constructor-default attention
(location features, softmax, no forward attention) and for the location + forward + transition-agent
config, L = 100 (multi-launch path: the resident decoder serves the synthesis configuration only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import load_pkg, weights_mod  # noqa: E402

t2 = load_pkg("tacotron2")
ids = torch.from_numpy(weights_mod().synthetic_ids(100, 1))[None]
for name, kw in (("loc_softmax", dict(attn_norm="softmax", forward_attn=False, location_attn=True)),
                 ("loc_fwd_ta", dict(attn_norm="sigmoid", forward_attn=True, trans_agent=True, location_attn=True))):
    m = t2.Tacotron2(130, 0, r=1, **kw).cuda().eval()
    m.decoder.max_decoder_steps = 300
    for _ in range(2):
        m.inference(ids)
    t = m.last_timing
    k = m.profile_step_kernels(reps=50)
    print(name, {"loop_ms": round(t["decoder_loop_ms"], 3), "steps": t["decoder_steps_run"],
                 "resident": t["resident"]}, {a: round(b * 1e3, 2) for a, b in k.items()})
