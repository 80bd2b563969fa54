"""Measurement (GPU box): one batched Griffin-Lim run (B = 8 ragged sentences, 10 iterations, the
per-iteration overlap-add + wave launches) saved to argv[1], so two libraries (TTS_HIP_LIB) can be
compared bitwise: python tools/gl_batch_bits.py out.npy [b1]  (b1: one 222-frame sentence, 60
iterations: the persistent loop)"""
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from conftest import load_pkg, tacotron2_config  # noqa: E402

audio = load_pkg("audio")
b1 = len(sys.argv) > 2 and sys.argv[2] == "b1"
ap = audio.AudioProcessor(**{**tacotron2_config()["audio"], "griffin_lim_iters": 60 if b1 else 10})
rng = np.random.Generator(np.random.PCG64(5))
lens = [222] if b1 else [200, 150, 173, 90, 201, 64, 120, 199]
mel = torch.from_numpy(rng.uniform(0, 1, size=(len(lens), max(lens), 80)).astype(np.float32)).cuda()
pu = rng.uniform(0, 1, size=(len(lens), 1025, max(lens)))
w = ap.griffin_lim_batch(mel, lens, phase_u=pu)
print(ap.last_gl_path())
np.save(sys.argv[1], w.cpu().numpy())
