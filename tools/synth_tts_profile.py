"""Synthesizer.tts() at the server configuration (config_tacotron2.json: mask off, 3000-step cap),
1- and N-sentence requests, for a rocprofv3 kernel trace of the whole drop-in call (GPU box helper):

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tts -- python3 tools/synth_tts_profile.py --n 1

Prints the wall time of each request (host work included)."""
import argparse
import importlib
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
gu = importlib.import_module("your-voice-tts_amd.generic_utils")
weights = importlib.import_module("your-voice-tts_amd.weights")
audiomod = importlib.import_module("your-voice-tts_amd.audio")
synth = importlib.import_module("your-voice-tts_amd.synthesis")

SENTENCES = ["It took me quite a long time to develop a voice.", "Now that I have it I am not going to be silent.",
             "Dr. Smith spoke to the crowd for an hour!", "Then we all went home?", "The rain kept falling.",
             "Nobody knew why the lights went out.", "We waited in the dark for a while.", "Then the music began."]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="1,4", help="sentences per request")
    ap.add_argument("--L", type=int, default=100)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    cfg = gu.default_config("config_tacotron2.json")
    m = gu.setup_model(130, cfg, max_batch=8, max_len=256)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in weights.tacotron2_weights(0).items()})
    m.decoder.max_decoder_steps = 3000
    m = m.cuda().eval()
    audio = dict(cfg.audio)
    audio["griffin_lim_iters"] = 60
    ap_ = audiomod.AudioProcessor(**audio)
    table = {s: weights.synthetic_ids(args.L, 1 + k) for k, s in enumerate(SENTENCES)}
    s = synth.Synthesizer(m, ap_, cfg, input_adapter=lambda sen: table[sen])
    for n in [int(x) for x in args.n.split(",")]:
        text = " ".join(SENTENCES[:n])
        np.random.seed(0)
        s.tts(text)
        for r in range(args.reps):
            np.random.seed(r)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            buf = s.tts(text)
            print(f"n={n} rep={r} wall_ms={1000 * (time.perf_counter() - t0):.2f} bytes={len(buf.getvalue())} "
                  f"decoder={m.last_timing.get('resident_kind')}", flush=True)


if __name__ == "__main__":
    main()
