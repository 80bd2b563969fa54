"""Measurement (GPU box): the Griffin-Lim implementation's own error against the oracle on the SAME
mel input and phases (no model noise): relative RMS of the GPU waveform vs AudioOracle's
inv_mel_spectrogram, for the reference-run configs[1] mel_post (222 frames: the one-per-CU
persistent form) and the sens_t342 float64 mel_post (342 frames: the two-per-CU form), over a few
phase draws.  Run once per library (TTS_HIP_LIB) to compare implementations.

    python tools/gl_accuracy.py
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from conftest import golden, load_pkg, rel_rms, tacotron2_config  # noqa: E402
from oracle.griffin_lim_oracle import AudioOracle  # noqa: E402

audio_cfg = tacotron2_config()["audio"]
ap = load_pkg("audio").AudioProcessor(**audio_cfg)
ao = AudioOracle(**audio_cfg)
res = {}
for name, mel in (("t222", golden("t2_fwdmask_L100")["mel_post"]), ("t342", golden("sens_t342")["mel_post64"])):
    mel = np.asarray(mel, np.float32)
    T = mel.shape[0]
    errs = []
    for seed in range(4):
        pu = np.random.Generator(np.random.PCG64(100 + seed)).uniform(0, 1, size=(1, 1025, T))
        wav = ap.griffin_lim_batch(torch.from_numpy(mel[None]).cuda(), [T], phase_u=pu).cpu().numpy()[0]
        ref = ao.inv_mel_spectrogram(mel.T, pu[0])
        errs.append(rel_rms(wav, ref))
    res[name] = dict(path=ap.last_gl_path(), rel_rms=errs, mean=float(np.mean(errs)))
    print(name, res[name], flush=True)
print(json.dumps(res))
