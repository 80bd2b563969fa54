"""Resident TacotronGST decoder: decoder-loop time and per-phase µs per step on a config-5 batch
(B=32 by default, L ~ U{60..160} seed 4, speakers b mod 4, style mel seed 4).  Measurement only."""
import importlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gu = importlib.import_module("your-voice-tts_amd.generic_utils")
weights = importlib.import_module("your-voice-tts_amd.weights")


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    cfg = gu.default_config("config_tacotron_gst.json")
    m = gu.setup_model(130, 4, cfg).cuda().eval()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in weights.tacotron_gst_weights(0, num_speakers=4).items()})
    lens = weights.synthetic_lengths(B, 4)
    ids = [weights.synthetic_ids(int(L), 200 + b) for b, L in enumerate(lens)]
    style = torch.from_numpy(np.random.Generator(np.random.PCG64(4)).uniform(0, 1, size=(B, 200, 80)).astype(np.float32))
    spk = [b % 4 for b in range(B)]
    for _ in range(3):
        out = m.inference_batch(ids, speaker_ids=spk, style_mel=style, postnet=False)
        torch.cuda.synchronize()
        lt = dict(m.last_timing)
        print(json.dumps(dict(loop_ms=lt["decoder_loop_ms"], steps=lt["decoder_steps_run"], resident=lt["resident"],
                              us_per_step=1000 * lt["decoder_loop_ms"] / max(1, lt["decoder_steps_run"]))))
    if lt["resident"]:
        ph = m.profile_resident_phases()
        for cu, d in ph.items():
            print(cu, "total %.2f" % sum(d.values()), json.dumps({k: round(v, 2) for k, v in d.items()}))


if __name__ == "__main__":
    main()
