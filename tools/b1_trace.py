"""configs[1] sentences through tts_synth_run for a kernel trace (measurement only):
python tools/b1_trace.py [sync] -- 20 sentences, pipelined unless 'sync'."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import load_pkg, weights_mod  # noqa: E402

sync = len(sys.argv) > 1 and sys.argv[1] == "sync"
gu = load_pkg("generic_utils")
audio = load_pkg("audio")
cfg = gu.default_config("config_tacotron2.json")
cfg.forward_attn_mask = True
m = gu.setup_model(130, cfg, max_batch=1, max_len=256).cuda().eval()
ap = audio.AudioProcessor(**cfg.audio)
ids = weights_mod().synthetic_ids(100, 1)
for k in range(25):
    m.synthesize_native([ids], ap, seed=k, sync=sync)
m.synth_sync()
torch.cuda.synchronize()
print("done")
