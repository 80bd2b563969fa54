"""Profiling target (tools only): one batched Griffin-Lim call (B=64, configs[2]-like frame counts,
random mels) on the default iteration kernel, after one warm-up call."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import load_pkg  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
audio = load_pkg("audio")
cfg = load_pkg("generic_utils").default_config("config_tacotron2.json")
rng = np.random.Generator(np.random.PCG64(2))
Fs = [int(2 * L + 22) for L in rng.integers(60, 161, size=B)]
mel = torch.from_numpy(rng.uniform(0, 1, size=(B, max(Fs), 80)).astype(np.float32)).cuda()
ap = audio.AudioProcessor(**cfg.audio)
for _ in range(2):
    ap.griffin_lim_batch(mel, Fs, seed=3, iters=int(os.environ.get("GL_ITERS", "10")))
torch.cuda.synchronize()
print("ok", sum(Fs))
