"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py) — Griffin-Lim path restated on the CPU.

Restates ``AudioProcessor`` (reference ``utils/audio.py``) and the librosa 0.6.2 functions it
calls.  librosa==0.6.2 is the version pinned by the reference (``setup.py:77``); it is not
installed in this image, so the librosa functions below are restated from its published
algorithm and their parity is UNPINNED (no reference test holds GL values:
``tests/test_audio.py:23-55`` only writes wav files).  Precision follows the reference: the
STFT matrix is stored complex64, the iSTFT accumulates float64 frames into a float32 signal,
the linear magnitude is float64 and the inverse pre-emphasis output is float64.
"""
from __future__ import annotations

import numpy as np
import scipy.fftpack as fftpack
import scipy.signal

# ---------------------------------------------------------------- librosa 0.6.2 restatement


def hann_periodic(n: int) -> np.ndarray:
    """``scipy.signal.get_window('hann', n, fftbins=True)`` (librosa ``filters.get_window``)."""
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)


def pad_center(w: np.ndarray, size: int) -> np.ndarray:
    """librosa ``util.pad_center``: lpad = (size - n) // 2, zeros on both sides."""
    n = len(w)
    lpad = (size - n) // 2
    return np.pad(w, (lpad, size - n - lpad), mode="constant")


def _hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if f.ndim:
        t = f >= min_log_hz
        mels[t] = min_log_mel + np.log(f[t] / min_log_hz) / logstep
    elif f >= min_log_hz:
        mels = min_log_mel + np.log(f / min_log_hz) / logstep
    return mels


def _mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if m.ndim:
        t = m >= min_log_mel
        freqs[t] = min_log_hz * np.exp(logstep * (m[t] - min_log_mel))
    elif m >= min_log_mel:
        freqs = min_log_hz * np.exp(logstep * (m - min_log_mel))
    return freqs


def mel_filters(sr, n_fft, n_mels=128, fmin=0.0, fmax=None):
    """librosa 0.6.2 ``filters.mel`` (Slaney mel scale, htk=False, norm=1 area normalisation)."""
    if fmax is None:
        fmax = float(sr) / 2
    weights = np.zeros((n_mels, 1 + n_fft // 2))
    fftfreqs = np.linspace(0, float(sr) / 2, 1 + n_fft // 2, endpoint=True)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights


def _frame(y, frame_length, hop_length):
    n_frames = 1 + int((len(y) - frame_length) / hop_length)
    idx = np.arange(frame_length)[:, None] + hop_length * np.arange(n_frames)[None, :]
    return y[idx]


def stft(y, n_fft=2048, hop_length=None, win_length=None, center=True):
    """librosa 0.6.2 ``stft``: periodic Hann padded to n_fft, reflect pad n_fft//2,
    scipy.fftpack FFT per frame, complex64 result [1 + n_fft//2, n_frames]."""
    if win_length is None:
        win_length = n_fft
    if hop_length is None:
        hop_length = win_length // 4
    if not np.issubdtype(y.dtype, np.floating) or y.ndim != 1 or not np.all(np.isfinite(y)):
        raise ValueError("invalid audio buffer")
    win = pad_center(hann_periodic(win_length), n_fft).reshape(-1, 1)
    if center:
        y = np.pad(y, n_fft // 2, mode="reflect")
    frames = _frame(y, n_fft, hop_length)
    spec = fftpack.fft(win * frames, axis=0)[: 1 + n_fft // 2]
    return spec.astype(np.complex64)


def window_sumsquare(n_frames, hop_length, win_length, n_fft, dtype=np.float32):
    """librosa 0.6.2 ``filters.window_sumsquare`` for the Hann window, norm=None."""
    n = n_fft + hop_length * (n_frames - 1)
    x = np.zeros(n, dtype=dtype)
    win_sq = pad_center(hann_periodic(win_length) ** 2, n_fft)
    for i in range(n_frames):
        s = i * hop_length
        x[s:min(n, s + n_fft)] += win_sq[: max(0, min(n_fft, n - s))]
    return x


def istft(stft_matrix, hop_length=None, win_length=None, center=True, dtype=np.float32):
    """librosa 0.6.2 ``istft``: per-frame inverse FFT of the Hermitian-extended spectrum,
    windowed, overlap-added into a float32 signal, divided by the window sum-square where it
    exceeds ``tiny``, trimmed by n_fft//2 on both sides."""
    n_fft = 2 * (stft_matrix.shape[0] - 1)
    if win_length is None:
        win_length = n_fft
    if hop_length is None:
        hop_length = win_length // 4
    win = pad_center(hann_periodic(win_length), n_fft)
    n_frames = stft_matrix.shape[1]
    y = np.zeros(n_fft + hop_length * (n_frames - 1), dtype=dtype)
    full = np.concatenate((stft_matrix, stft_matrix[-2:0:-1].conj()), axis=0)
    frames = win[:, None] * fftpack.ifft(full, axis=0).real  # float64 [n_fft, n_frames]
    for i in range(n_frames):  # sequential float32 accumulation, frame order as librosa
        s = i * hop_length
        y[s:s + n_fft] = y[s:s + n_fft] + frames[:, i]
    wss = window_sumsquare(n_frames, hop_length, win_length, n_fft, dtype=dtype)
    nz = wss > np.finfo(wss.dtype).tiny
    y[nz] /= wss[nz]
    if center:
        y = y[n_fft // 2: -(n_fft // 2)]
    return y


def device_phase_u(seed: int, b: int, F: int, nb: int = 1025) -> np.ndarray:
    """The U[0,1) initial phases the HIP Griffin-Lim draws on the device when no host phases are
    given (griffin_lim.hip: hash_uniform, a splitmix64 finaliser of seed + golden * (idx + 1) with
    idx = (b * 1025 + k) * 2^20 + f), restated with wrapping uint64 arithmetic: [nb, F] float64."""
    with np.errstate(over="ignore"):
        k = np.arange(nb, dtype=np.uint64)[:, None]
        f = np.arange(F, dtype=np.uint64)[None, :]
        idx = (np.uint64(b) * np.uint64(nb) + k) * np.uint64(1048576) + f
        z = np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15) * (idx + np.uint64(1))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


# ---------------------------------------------------------------- AudioProcessor restatement


class AudioOracle:
    """Restates the inverse half of ``AudioProcessor`` (reference ``utils/audio.py:11-201``)."""

    def __init__(self, sample_rate=22050, num_mels=80, min_level_db=-100, frame_shift_ms=12.5,
                 frame_length_ms=50, ref_level_db=20, num_freq=1025, power=1.5,
                 preemphasis=0.98, signal_norm=True, symmetric_norm=False, max_norm=1.0,
                 mel_fmin=0.0, mel_fmax=8000.0, clip_norm=True, griffin_lim_iters=60, **_):
        self.sample_rate = sample_rate
        self.num_mels = num_mels
        self.min_level_db = min_level_db
        self.ref_level_db = ref_level_db
        self.num_freq = num_freq
        self.power = power
        self.preemphasis = preemphasis
        self.signal_norm = signal_norm
        self.symmetric_norm = symmetric_norm
        self.max_norm = 1.0 if max_norm is None else float(max_norm)
        self.clip_norm = clip_norm
        self.mel_fmin = 0 if mel_fmin is None else mel_fmin
        self.mel_fmax = mel_fmax
        self.griffin_lim_iters = griffin_lim_iters
        # utils/audio.py:114-119
        self.n_fft = (num_freq - 1) * 2
        self.hop_length = int(frame_shift_ms / 1000.0 * sample_rate)
        self.win_length = int(frame_length_ms / 1000.0 * sample_rate)

    def mel_basis(self):  # utils/audio.py:68-77
        return mel_filters(self.sample_rate, self.n_fft, self.num_mels, self.mel_fmin, self.mel_fmax)

    def denormalize(self, S):  # utils/audio.py:96-112
        if not self.signal_norm:
            return S
        if self.symmetric_norm:
            if self.clip_norm:
                S = np.clip(S, -self.max_norm, self.max_norm)
            return ((S + self.max_norm) * -self.min_level_db / (2 * self.max_norm)) + self.min_level_db
        if self.clip_norm:
            S = np.clip(S, 0, self.max_norm)
        return (S * -self.min_level_db / self.max_norm) + self.min_level_db

    @staticmethod
    def db_to_amp(x):  # utils/audio.py:125-126
        return np.power(10.0, x * 0.05)

    def mel_to_linear(self, mel):  # utils/audio.py:64-66
        return np.maximum(1e-10, np.dot(np.linalg.pinv(self.mel_basis()), mel))

    def inv_preemphasis(self, x):  # utils/audio.py:133-136
        if self.preemphasis == 0:
            raise RuntimeError(" !! Preemphasis is applied with factor 0.0. ")
        return scipy.signal.lfilter([1], [1, -self.preemphasis], x)

    def griffin_lim(self, S, phase_u=None, iters=None):  # utils/audio.py:182-189
        """``phase_u``: the U[0,1) draws the reference takes from ``np.random.rand``."""
        if phase_u is None:
            phase_u = np.random.rand(*S.shape)
        iters = self.griffin_lim_iters if iters is None else iters
        angles = np.exp(2j * np.pi * phase_u)
        S_complex = np.abs(S).astype(np.complex128)
        y = istft(S_complex * angles, self.hop_length, self.win_length)
        for _ in range(iters):
            angles = np.exp(1j * np.angle(stft(y, self.n_fft, self.hop_length, self.win_length)))
            y = istft(S_complex * angles, self.hop_length, self.win_length)
        return y

    def mel_magnitude(self, mel):
        """mel [80,T] -> linear magnitude ** power [1025,T] float64 (utils/audio.py:166-170)."""
        S = self.db_to_amp(self.denormalize(mel) + self.ref_level_db)
        return self.mel_to_linear(S) ** self.power

    def linear_magnitude(self, spec):
        """linear [1025,T] -> magnitude ** power (utils/audio.py:156-160)."""
        S = self.db_to_amp(self.denormalize(spec) + self.ref_level_db)
        return S ** self.power

    def inv_mel_spectrogram(self, mel, phase_u=None, iters=None):  # utils/audio.py:164-172
        y = self.griffin_lim(self.mel_magnitude(mel), phase_u, iters)
        return self.inv_preemphasis(y) if self.preemphasis != 0 else y

    def inv_spectrogram(self, spec, phase_u=None, iters=None):  # utils/audio.py:154-162
        y = self.griffin_lim(self.linear_magnitude(spec), phase_u, iters)
        return self.inv_preemphasis(y) if self.preemphasis != 0 else y

    # ---- forward half used by compute_style_mel (utils/synthesis.py:28-35)
    def apply_preemphasis(self, x):  # utils/audio.py:128-131
        if self.preemphasis == 0:
            raise RuntimeError(" !! Preemphasis is applied with factor 0.0. ")
        return scipy.signal.lfilter([1, -self.preemphasis], [1], x)

    def amp_to_db(self, x):  # utils/audio.py:121-123
        min_level = np.exp(self.min_level_db / 20 * np.log(10))
        return 20 * np.log10(np.maximum(min_level, x))

    def normalize(self, S):  # utils/audio.py:79-94
        if not self.signal_norm:
            return S
        S_norm = (S - self.min_level_db) / -self.min_level_db
        if self.symmetric_norm:
            S_norm = (2 * self.max_norm) * S_norm - self.max_norm
            return np.clip(S_norm, -self.max_norm, self.max_norm) if self.clip_norm else S_norm
        S_norm = self.max_norm * S_norm
        return np.clip(S_norm, 0, self.max_norm) if self.clip_norm else S_norm

    def melspectrogram(self, y):  # utils/audio.py:146-152
        y = self.apply_preemphasis(y) if self.preemphasis != 0 else y
        D = stft(y, self.n_fft, self.hop_length, self.win_length)
        S = self.amp_to_db(np.dot(self.mel_basis(), np.abs(D))) - self.ref_level_db
        return self.normalize(S)

    @staticmethod
    def wav_to_int16(wav):  # utils/audio.py:56-58 (the value save_wav writes)
        wav = np.asarray(wav)
        return (wav * (32767 / max(0.01, np.max(np.abs(wav))))).astype(np.int16)
