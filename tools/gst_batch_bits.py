"""Measurement (GPU box): one TacotronGST batch (B = 32, config-5 shaped, 200-step cap) whose
linear spectrogram is saved to argv[1], so two libraries or knob settings can be compared
bitwise: python tools/gst_batch_bits.py out.npy"""
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from conftest import load_pkg, weights_mod  # noqa: E402

w = weights_mod()
gu = load_pkg("generic_utils")
cfg = gu.default_config("config_tacotron_gst.json")
lens = w.synthetic_lengths(32, 4)
ids = [w.synthetic_ids(int(L), 300 + b) for b, L in enumerate(lens)]
style = torch.from_numpy(np.random.Generator(np.random.PCG64(8)).uniform(0, 1, size=(32, 200, 80)).astype(np.float32))
m = gu.setup_model(130, 4, cfg).cuda().eval()
m.decoder.max_decoder_steps = 200
out = m.inference_batch(ids, speaker_ids=[b % 4 for b in range(32)], style_mel=style)
print("frames", sum(out["frames"]))
np.save(sys.argv[1], out["linear"].cpu().numpy())
