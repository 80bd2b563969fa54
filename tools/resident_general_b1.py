"""Measurement only: batch-1 decoder loop per attention configuration at L = 100, the resident
decoder (general form for every configuration but synthesize.py's masked one) against the
multi-launch path (TTS_RESIDENT_GEN=0 / TTS_RESIDENT=0 at create).  µs per step from the decoder's
own HIP-event loop timer (tts_decoder_last_timing), median of 5 calls after 2 warm-up calls.
Writes one JSON object to stdout (and to argv[1] when given)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import load_pkg, weights_mod  # noqa: E402

t2 = load_pkg("tacotron2")
ids = torch.from_numpy(weights_mod().synthetic_ids(100, 1))[None]
CONFIGS = {
    # Synthesizer.tts(): config_tacotron2.json as is (server/synthesizer.py:46-66), 3000-step cap
    "server_fwd_sigmoid_nomask": (dict(attn_norm="sigmoid", forward_attn=True, forward_attn_mask=False,
                                       location_attn=False), 3000),
    # synthesize.py:86 (the headline path, mask form)
    "synthesize_fwd_sigmoid_mask": (dict(attn_norm="sigmoid", forward_attn=True, forward_attn_mask=True,
                                         location_attn=False), 1000),
    # models/tacotron2.py:17,23 constructor default
    "default_loc_softmax": (dict(attn_norm="softmax", forward_attn=False, location_attn=True), 1000),
    "loc_fwd_ta": (dict(attn_norm="sigmoid", forward_attn=True, trans_agent=True, location_attn=True), 1000),
    "win_softmax": (dict(attn_norm="softmax", forward_attn=False, location_attn=False, attn_win=True), 1000),
}


def run(kw, cap, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        m = t2.Tacotron2(130, 0, r=1, **kw)
        m.decoder.max_decoder_steps = cap
        m = m.cuda().eval()
        m.inference(ids)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    m.inference(ids)
    per = []
    for _ in range(5):
        m.inference(ids)
        t = m.last_timing
        per.append(1e3 * t["decoder_loop_ms"] / t["decoder_steps_run"])
    return dict(us_per_step=round(statistics.median(per), 3), steps=t["decoder_steps_run"],
                resident=bool(t["resident"]))


out = {}
only = [c for c in os.environ.get("TTS_CONFIGS", "").split(",") if c]
for name, (kw, cap) in CONFIGS.items():
    if only and name not in only:
        continue
    out[name] = {"resident": run(kw, cap, {"TTS_RESIDENT_GEN": "1"})}
    if not os.environ.get("TTS_NO_ML"):  # (A/B runs of the resident forms skip the multi-launch leg)
        out[name]["multi_launch"] = run(kw, cap, {"TTS_RESIDENT_GEN": "0", "TTS_RESIDENT": "0"})
    print(name, out[name], flush=True)
res = {"workload": "batch 1, L=100 (synthetic ids seed 1), decoder loop only", "configs": out}
print(json.dumps(res))
if len(sys.argv) > 1:
    json.dump(res, open(sys.argv[1], "w"), indent=1)
