"""CPU: the C-ABI library loads and exports every symbol include/tts_hip.h declares; the
product path refuses to run without a GPU (no CPU fallback).  No compute calls here."""
import os
import re
import subprocess

import pytest
import torch

from conftest import REPO, load_pkg

HEADER = os.path.join(REPO, "include", "tts_hip.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(tts_[a-z0-9_]+)\s*\(", txt)))


def test_header_matches_binding_table():
    n = load_pkg("_native")
    assert header_symbols() == sorted(n.EXPORTS)


def test_library_exports_every_header_symbol():
    n = load_pkg("_native")
    lib = n.load_library()
    for s in header_symbols():
        assert hasattr(lib, s), s
    assert lib.tts_version().startswith(b"libtts_hip")
    out = subprocess.run(["nm", "-D", "--defined-only", n.LIB_PATH], capture_output=True, text=True).stdout
    for s in header_symbols():
        assert re.search(r"\bT " + s + r"\b", out), s


def test_library_targets_gfx950():
    n = load_pkg("_native")
    data = open(n.LIB_PATH, "rb").read()
    assert b"gfx950" in data


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_no_cpu_fallback():
    t2 = load_pkg("tacotron2")
    m = t2.Tacotron2(130, 0, r=1, attn_norm="sigmoid", forward_attn=True, forward_attn_mask=True,
                     location_attn=False)
    with pytest.raises(RuntimeError, match="no GPU"):
        m.inference(torch.arange(3, 20)[None])
    audio = load_pkg("audio")
    ap = audio.AudioProcessor(**load_pkg("generic_utils").default_config()["audio"])
    with pytest.raises(RuntimeError, match="no GPU"):
        ap.inv_mel_spectrogram(torch.rand(80, 10).numpy())


def test_speaker_ids_must_match_the_batch():
    """the library reads B speaker ids; one id broadcasts, any other count is rejected
    before the call (torch's broadcast add in models/tacotron2.py:91-100 rejects it too)."""
    t2 = load_pkg("tacotron2")
    assert t2._speaker_array(torch.tensor([3]), 4).tolist() == [3, 3, 3, 3]
    assert t2._speaker_array([0, 1, 2], 3).tolist() == [0, 1, 2]
    with pytest.raises(ValueError):
        t2._speaker_array([0, 1], 3)
    with pytest.raises(ValueError):
        t2._speaker_array([0, 1, 2, 3], 3)
