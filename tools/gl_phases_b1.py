import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import load_pkg
audio = load_pkg("audio"); cfg = load_pkg("generic_utils").default_config("config_tacotron2.json")
rng = np.random.Generator(np.random.PCG64(2))
F = int(os.environ.get("GL_F", "222"))  # frame count (above 256: the two-per-CU persistent form)
mel = torch.from_numpy(rng.uniform(0, 1, size=(1, F, 80)).astype(np.float32)).cuda()
ap = audio.AudioProcessor(**cfg.audio)
for k in range(3):
    ap.griffin_lim_batch(mel, [F], seed=3)
torch.cuda.synchronize()
print(ap.last_gl_path(), ap.last_gl_timing())
