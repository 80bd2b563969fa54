"""Measurement only: the configs[2]-shaped B=64 decoder as one handle vs two B=32 handles driven
concurrently from two host threads on two streams (does the second batch fill the first one's
launch gaps?).  Prints one JSON line."""
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.conftest import load_pkg  # noqa: E402

w = load_pkg("weights")
t2 = load_pkg("tacotron2")
FL = dict(attn_win=False, attn_norm="sigmoid", forward_attn=True, trans_agent=False, forward_attn_mask=True,
          location_attn=False)
lens = [int(x) for x in w.synthetic_lengths(64, 2)]
ids = [w.synthetic_ids(L, 100 + b) for b, L in enumerate(lens)]


def model(B):
    m = t2.Tacotron2(130, 0, r=1, max_batch=B, **FL)
    m.decoder.max_decoder_steps = 1000
    return m.cuda().eval()


m0 = model(64)
Lmax = max(lens)
idt = torch.zeros(64, Lmax, dtype=torch.long)
for b, x in enumerate(ids):
    idt[b, :lens[b]] = torch.as_tensor(x)
enc = m0.encode(idt.cuda(), lens)
order = sorted(range(64), key=lambda b: lens[b])
halves = [order[0::2], order[1::2]]
encs = [enc[h].contiguous() for h in halves]
lhs = [[lens[b] for b in h] for h in halves]
ms = [model(32), model(32)]
streams = [torch.cuda.Stream(), torch.cuda.Stream()]


def one():
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = m0.inference_batch(None, enc=enc, lens=lens)
    torch.cuda.synchronize()
    return time.perf_counter() - t, out["steps"]


def two(serial=False):
    res = [None, None]

    def run(i):
        with torch.cuda.stream(streams[i]):
            res[i] = ms[i].inference_batch(None, enc=encs[i], lens=lhs[i])["steps"]
        streams[i].synchronize()

    torch.cuda.synchronize()
    t = time.perf_counter()
    if serial:
        run(0)
        run(1)
    else:
        th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    torch.cuda.synchronize()
    return time.perf_counter() - t, res


for _ in range(2):
    one(), two(), two(True)
r = {"one_b64_ms": [], "two_b32_concurrent_ms": [], "two_b32_serial_ms": []}
for _ in range(3):
    a, s0 = one()
    b, s2 = two()
    c, _ = two(True)
    r["one_b64_ms"].append(round(a * 1e3, 2))
    r["two_b32_concurrent_ms"].append(round(b * 1e3, 2))
    r["two_b32_serial_ms"].append(round(c * 1e3, 2))
r["max_steps"] = max(s0)
r["same_steps"] = sorted(s0) == sorted(s2[0] + s2[1])
print(json.dumps(r))
