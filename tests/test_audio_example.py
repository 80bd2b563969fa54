"""The reference's only natural-speech input: tests/inputs/example_1.wav through
tests/test_audio.py:23-55 (melspectrogram -> inv_mel_spectrogram at ten normalisation settings of
tests/test_config.json), replayed on the reference's own AudioProcessor by
tests/golden/make_golden.py (audio_example1.npz; librosa 0.6.2 restated, its internals unpinned).

Every other Griffin-Lim check runs on random-weight mels, half of them clipped to the floor; this is
phase retrieval on a real harmonic spectrum.  CPU: the oracle restatement against the fixture.
GPU: the HIP mel analysis (tts_gl_melspectrogram) and the HIP Griffin-Lim (30 iterations, the
test config's count, phases from numpy's stream seeded as the fixture was) against it.
"""
import ast

import numpy as np
import pytest

from conftest import golden, load_pkg, rel_rms
from oracle.griffin_lim_oracle import AudioOracle

Z = golden("audio_example1")
SETTINGS = [tuple(s) for s in Z["settings"]]
WAV_RTOL = 1e-4  # north_star's waveform tolerance (GL amplifies fp32 rounding ~100x)


def _cfg(i):
    audio = ast.literal_eval(str(Z["audio"]))
    max_norm, signal_norm, symmetric_norm, clip_norm = SETTINGS[i]
    return {**audio, "max_norm": max_norm, "signal_norm": bool(signal_norm),
            "symmetric_norm": bool(symmetric_norm), "clip_norm": bool(clip_norm)}


def _x():
    return Z["pcm"].astype(np.float64) / 32768.0  # soundfile's float64 read of int16 PCM


def _mel_tol(ref):
    return 1e-5 * max(1.0, float(np.abs(ref).max()))  # float32 output; dB units without signal_norm


@pytest.mark.parametrize("i", range(10))
def test_oracle_melspectrogram_matches_reference(i):
    mel = AudioOracle(**_cfg(i)).melspectrogram(_x())
    assert mel.shape == Z[f"mel{i}"].shape
    assert np.abs(mel - Z[f"mel{i}"]).max() <= 1e-9 * max(1.0, float(np.abs(Z[f"mel{i}"]).max()))


@pytest.mark.parametrize("i", [0, 4, 9])
def test_oracle_griffin_lim_matches_reference(i):
    o = AudioOracle(**_cfg(i))
    mel = Z[f"mel{i}"]
    np.random.seed(1000 + i)
    wav = o.inv_mel_spectrogram(mel, phase_u=np.random.rand(o.n_fft // 2 + 1, mel.shape[1]))
    assert wav.shape == Z[f"wav{i}"].shape
    assert rel_rms(wav, Z[f"wav{i}"]) < 1e-6  # (the fixture is stored float32)


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(10))
def test_gpu_melspectrogram_example_wav(i):
    ap = load_pkg("audio").AudioProcessor(**_cfg(i))
    ref = Z[f"mel{i}"]
    mel = ap.melspectrogram(_x())
    assert mel.shape == ref.shape
    assert np.abs(mel - ref).max() <= _mel_tol(ref)


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(10))
def test_gpu_griffin_lim_example_wav(i):
    """inv_mel_spectrogram (utils/audio.py:164-172) of the reference's mel: HIP magnitude, 30 GL
    iterations, de-emphasis; phases from numpy's stream (np.random.seed(1000 + i), as the fixture)."""
    ap = load_pkg("audio").AudioProcessor(**_cfg(i))
    np.random.seed(1000 + i)
    wav = ap.inv_mel_spectrogram(Z[f"mel{i}"])
    assert wav.shape == Z[f"wav{i}"].shape
    assert rel_rms(wav, Z[f"wav{i}"]) < WAV_RTOL, i
