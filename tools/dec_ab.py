"""A/B helper (GPU box): median decoder-loop time per step of the batch-1 resident decoder on
configs[1]'s sentence for the library named by TTS_HIP_LIB (measurement only)."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
from conftest import golden_flags, golden, load_pkg, weights_mod  # noqa: E402

gu = load_pkg("generic_utils")
cfg = gu.default_config("config_tacotron2.json")
cfg.forward_attn_mask = True
m = gu.setup_model(130, cfg, max_batch=1, max_len=256).cuda().eval()
ids = weights_mod().synthetic_ids(100, 1)
ts = []
for k in range(40):
    out = m.inference_batch([ids])
    if k >= 5:
        ts.append(m.last_timing["decoder_loop_ms"] * 1000 / out["steps"][0])
torch.cuda.synchronize()
print(json.dumps(dict(us_per_step=float(np.median(ts)), p10=float(np.percentile(ts, 10)),
                      p90=float(np.percentile(ts, 90)), resident=m.last_timing["resident"], steps=out["steps"][0])))
