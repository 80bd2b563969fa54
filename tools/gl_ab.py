"""GPU A/B of the batched Griffin-Lim iteration kernels (tools only, not a test): B sentences of
random mels at configs[2]-like lengths; per-kernel mean time from tts_gl_profile for the wave
kernel (default) and the 256-thread block kernel (TTS_GL_WAVE=0), plus their waveform agreement."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import load_pkg  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    audio = load_pkg("audio")
    gu = load_pkg("generic_utils")
    cfg = gu.default_config("config_tacotron2.json")
    rng = np.random.Generator(np.random.PCG64(2))
    Fs = [int(2 * L + 22) for L in rng.integers(60, 161, size=B)]
    Fmax = max(Fs)
    mel = torch.from_numpy(rng.uniform(0, 1, size=(B, Fmax, 80)).astype(np.float32)).cuda()
    out = {}
    for wave in ("1", "0"):
        os.environ["TTS_GL_WAVE"] = wave
        ap = audio.AudioProcessor(**cfg.audio)
        w = ap.griffin_lim_batch(mel, Fs, seed=3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            w = ap.griffin_lim_batch(mel, Fs, seed=3)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / 3 * 1e3
        prof = ap.profile_gl_kernels(10)
        out[wave] = w.cpu().numpy()
        print(f"TTS_GL_WAVE={wave} B={B} frames={sum(Fs)} path={ap.last_gl_path()} wall {wall:.2f} ms "
              f"loop {ap.last_gl_timing()['gl_loop_ms']:.2f} ms kernels(ms) {prof}", flush=True)
    d = out["1"] - out["0"]
    print("rel diff wave vs block", float(np.sqrt((d ** 2).mean() / (out["0"] ** 2).mean())))


if __name__ == "__main__":
    main()
