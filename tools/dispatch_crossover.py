"""Measurement only: a request of B sentences decoded as ONE batch on the
multi-launch path against B serial batch-1 calls on the resident decoder, B = 1..8, for the
Synthesizer.tts() configuration (config_tacotron2.json: forward attention, sigmoid, mask off, 3000-step
cap; server/synthesizer.py:46-66) and synthesize.py's (mask on).  Sentence lengths L ~ U{60..160}
(seed 5).  Wall time of the decode (Tacotron2 inference incl. encoder and postnet), median of 3 after a
warm-up; writes one JSON object (stdout, and argv[1] when given)."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import load_pkg, weights_mod  # noqa: E402

t2 = load_pkg("tacotron2")
w = weights_mod()
lens = [int(x) for x in w.synthetic_lengths(8, 5)]
ids = [w.synthetic_ids(L, 900 + i) for i, L in enumerate(lens)]
CONFIGS = {"server_nomask_cap3000": (dict(attn_norm="sigmoid", forward_attn=True, forward_attn_mask=False,
                                          location_attn=False), 3000),
           "synthesize_mask": (dict(attn_norm="sigmoid", forward_attn=True, forward_attn_mask=True,
                                    location_attn=False), 1000)}


def timed(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(1e3 * (time.perf_counter() - t0))
    return statistics.median(ts)


res = {}
for name, (kw, cap) in CONFIGS.items():
    m1 = t2.Tacotron2(130, 0, r=1, **kw)
    m1.decoder.max_decoder_steps = cap
    m1.max_len = 256
    m1 = m1.cuda().eval()
    mb = t2.Tacotron2(130, 0, r=1, **kw)
    mb.decoder.max_decoder_steps = cap
    mb.max_len, mb.max_batch = 256, 8
    mb = mb.cuda().eval()
    rows = []
    for B in range(1, 9):
        batch = ids[:B]
        serial = timed(lambda: [m1.inference_batch([x]) for x in batch])
        assert m1.last_timing["resident"]
        batched = timed(lambda: mb.inference_batch(batch))
        rows.append(dict(B=B, serial_resident_ms=round(serial, 3), batched_ms=round(batched, 3),
                         batched_resident=bool(mb.last_timing["resident"])))
        print(name, rows[-1], flush=True)
    res[name] = rows
    # whole requests (synthesize_batch: decode + one Griffin-Lim batch, 60 iterations) of 3 sentences,
    # dispatched serially (SERIAL_RESIDENT_MAX = 3, the default) and as one batch (0)
    synth = load_pkg("synthesis")
    import json as _j
    cfgd = _j.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                     "your-voice-tts_amd", "configs", "config_tacotron2.json")))
    ap = load_pkg("audio").AudioProcessor(**cfgd["audio"])
    req = {}
    for mx in (3, 0):
        synth.SERIAL_RESIDENT_MAX = mx
        info = {}

        def call():
            info.update(synth.synthesize_batch(mb, ap, ids[:3], seed=1)[1])
        req[f"serial_max_{mx}"] = dict(ms=round(timed(call), 3), dispatch=info["decoder_dispatch"])
    synth.SERIAL_RESIDENT_MAX = 3
    res[name + "_request3"] = req
    print(name, req, flush=True)
out = {"lengths": lens, "configs": res}
print(json.dumps(out))
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
