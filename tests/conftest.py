import ast
import importlib
import json
import os
import re
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)

PKG = "your-voice-tts_amd"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def load_pkg(sub=None):
    """Import the product package (its directory name is not an identifier)."""
    mod = importlib.import_module(PKG)
    return importlib.import_module(PKG + "." + sub) if sub else mod


def weights_mod():
    return load_pkg("weights")


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def golden_flags(z):
    return ast.literal_eval(str(z["flags"]))


def tacotron2_config():
    """config_tacotron2.json audio section (values as in the reference config, lines 5-25)."""
    return json.load(open(os.path.join(REPO, "your-voice-tts_amd", "configs", "config_tacotron2.json")))


def rel_rms(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(scope="session")
def audio_cfg():
    return tacotron2_config()["audio"]
