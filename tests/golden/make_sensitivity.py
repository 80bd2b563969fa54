"""Generates tests/golden/sens_t342.npz: the reference path's OWN numerical sensitivity at the
longest sentence of configs[3]'s per-rank share (L=160 -> T=342 frames).

The reference runs Tacotron2 in float32 (torch) and Griffin-Lim in float64 with float32 overlap-add
(librosa 0.6.2).  Any other correct fp32 implementation differs from it by float32 rounding in the
model, which the autoregressive decoder and 60 Griffin-Lim iterations then amplify.  This script
measures that amplification on the oracle (a numpy restatement of the reference, pinned by the
reference-run fixtures; no reference code runs here): the oracle chain in float32 vs the same chain
in float64, same ids, same weights (generator seed 0), same Griffin-Lim phases (device_phase_u seed
40, the row the sharded GPU test uses).  The float64 model output is kept as the high-precision
target for the GPU test; the numbers are the reference's noise floor the GPU tolerance is read
against.

    python tests/golden/make_sensitivity.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)

from conftest import golden, golden_flags, load_pkg, rel_rms, tacotron2_config, weights_mod  # noqa: E402
from oracle.griffin_lim_oracle import AudioOracle, device_phase_u  # noqa: E402
from oracle.tacotron2_oracle import Tacotron2Oracle  # noqa: E402

PHASE_SEED = 40


def configs3_longest():
    """(ids, index b in rank 0's batch) of the longest sentence of rank 0's LPT share of configs[3]."""
    w = weights_mod()
    sh = load_pkg("sharding")
    lens = w.synthetic_lengths(512, 3)
    ids = [w.synthetic_ids(int(L), 100 + b) for b, L in enumerate(lens)]
    mine = sh.lpt_partition([sh.sentence_cost(len(x), 1000) for x in ids], 8, capacity=64)[0]
    sub = [ids[i] for i in mine]
    b = int(np.argmax([len(x) for x in sub]))
    return sub[b], b


def measure():
    x, b = configs3_longest()
    fl = golden_flags(golden("t2_fwdmask_L100"))
    sd = weights_mod().tacotron2_weights(0)
    r32 = Tacotron2Oracle(sd, dtype=np.float32, **fl).inference(x)
    r64 = Tacotron2Oracle(sd, dtype=np.float64, **fl).inference(x)
    T = r32["mel"].shape[0]
    assert r64["mel"].shape[0] == T
    ao = AudioOracle(**tacotron2_config()["audio"])
    pu = device_phase_u(PHASE_SEED, b, T)
    w32 = ao.inv_mel_spectrogram(r32["mel_post"].T, pu)
    w64 = ao.inv_mel_spectrogram(r64["mel_post"].T, pu)
    return dict(ids=np.asarray(x, np.int64), b=b, phase_seed=PHASE_SEED,
                mel_post32=r32["mel_post"].astype(np.float32), mel_post64=r64["mel_post"],
                align_argmax64=r64["align"].argmax(1),
                mel_rel_32_64=rel_rms(r32["mel_post"], r64["mel_post"]), wav_rel_32_64=rel_rms(w32, w64))


if __name__ == "__main__":
    d = measure()
    np.savez_compressed(os.path.join(HERE, "sens_t342.npz"), **d)
    print({k: v for k, v in d.items() if np.ndim(v) == 0})
