"""CPU: the torch-CPU restatement (bench.py's cpu_baseline model half) against the reference's own
outputs (tests/golden/t2_*.npz), at the same bar as the numpy oracle."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden, golden_flags, rel_rms, weights_mod
from oracle.tacotron2_torch import Tacotron2TorchCPU

T2_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "t2_*.npz")))


@pytest.mark.parametrize("case", T2_CASES)
def test_torch_cpu_restatement_matches_reference(case):
    z = golden(case)
    fl = golden_flags(z)
    sd = weights_mod().tacotron2_weights(0, location_attn=fl["location_attn"], trans_agent=fl["trans_agent"])
    o = Tacotron2TorchCPU(sd, **fl)
    res = o.inference(z["ids"])
    assert rel_rms(res["enc"], z["enc"]) < 1e-5
    assert res["mel"].shape == z["mel"].shape, "frame count differs from the reference"
    np.testing.assert_array_equal(res["align"].argmax(1), z["align"].argmax(1))
    np.testing.assert_array_equal(res["stop"] > 0.5, z["stop"] > 0.5)
    assert rel_rms(res["mel"], z["mel"]) < 1e-4
    assert rel_rms(res["mel_post"], z["mel_post"]) < 1e-4
    assert np.abs(res["align"] - z["align"]).max() < 1e-4
