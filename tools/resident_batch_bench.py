"""Decoder loop time per step of the resident batch decoder (csrc/resident_batch.hip) against the
multi-launch batch and serial batch-1 resident calls, at the Synthesizer's configuration (mask off,
runs to the cap) and synthesize.py's (mask on).  GPU box helper; prints one JSON line per case.

    python tools/resident_batch_bench.py [--cap 1000] [--batches 2,3,4,8,12]
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
t2 = importlib.import_module("your-voice-tts_amd.tacotron2")
weights = importlib.import_module("your-voice-tts_amd.weights")


def model(mask, batch, cap):
    os.environ["TTS_RESIDENT_BATCH"] = "1" if batch else "0"
    m = t2.Tacotron2(130, 0, r=1, attn_norm="sigmoid", forward_attn=True, forward_attn_mask=mask,
                     location_attn=False, max_batch=16, max_len=256)
    m.decoder.max_decoder_steps = cap
    m = m.cuda().eval()
    m.inference_batch([[5, 6], [7, 8, 9]])
    return m


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cap", type=int, default=1000)
    ap.add_argument("--batches", default="2,3,4,8,12")
    ap.add_argument("--L", type=int, default=100)
    ap.add_argument("--mask", choices=("both", "on", "off"), default="both")
    ap.add_argument("--quick", action="store_true", help="the resident batch decoder only")
    args = ap.parse_args()
    for mask in {"both": (False, True), "on": (True,), "off": (False,)}[args.mask]:
        rb = model(mask, True, args.cap)
        ml = None if args.quick else model(mask, False, args.cap)
        for B in [int(x) for x in args.batches.split(",")]:
            ids = [weights.synthetic_ids(args.L, 1 + b) for b in range(B)]
            rec = dict(mask=mask, B=B, L=args.L, cap=args.cap)
            rec["resident_batch_ms"] = timed(lambda: rb.inference_batch(ids))
            rec["resident_kind"] = rb.last_timing.get("resident_kind")
            rec["decoder_loop_ms"] = rb.last_timing.get("decoder_loop_ms")
            steps = max(rb.inference_batch(ids)["steps"])
            rec["steps"] = steps
            rec["us_per_step"] = 1000 * rec["decoder_loop_ms"] / steps if steps else None
            if ml is not None:
                rec["multi_launch_ms"] = timed(lambda: ml.inference_batch(ids))
                rec["multi_launch_loop_ms"] = ml.last_timing.get("decoder_loop_ms")
                rec["serial_b1_ms"] = timed(lambda: [rb.inference_batch([x]) for x in ids], reps=1)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
