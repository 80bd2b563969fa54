"""Drop-in for the inverse half of the reference ``AudioProcessor`` (utils/audio.py:11-201).

``inv_mel_spectrogram`` / ``inv_spectrogram`` keep the reference signatures (numpy [n, T] in,
numpy float64 waveform out) and run Griffin-Lim on the GPU through libtts_hip ``tts_gl_run``:
denormalise -> dB->amp -> pinv(mel basis) -> ^power -> GL (librosa 0.6.2 stft/istft semantics)
-> inverse pre-emphasis, all in HIP.  The initial phases are drawn on the host with
``np.random.rand(*S.shape)`` exactly as utils/audio.py:183 does, so a caller that seeds numpy gets
the same phases as the reference.  ``inv_mel_spectrogram_batch`` is the batched GPU-resident form
(torch tensors in HBM, device-drawn phases) the batched/sharded synthesis uses.

The mel filter bank is librosa 0.6.2 ``filters.mel`` (Slaney, area-normalised), restated in
numpy because librosa is not installed; its pseudo-inverse is computed once in float64 on the
host (utils/audio.py:64-66 recomputes it on every call).
"""
from __future__ import annotations

import contextlib
import ctypes
import io as _io

import numpy as np
import scipy.io.wavfile
import scipy.signal
import torch

from . import _native


def _hz_to_mel(f):
    f = np.atleast_1d(np.asarray(f, dtype=np.float64))
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    mel = f / f_sp
    hi = f >= min_log_hz
    mel[hi] = min_log_mel + np.log(f[hi] / min_log_hz) / logstep
    return mel


def _mel_to_hz(m):
    m = np.atleast_1d(np.asarray(m, dtype=np.float64))
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    f = f_sp * m
    hi = m >= min_log_mel
    f[hi] = min_log_hz * np.exp(logstep * (m[hi] - min_log_mel))
    return f


def mel_basis(sr, n_fft, n_mels, fmin=0.0, fmax=None):
    """librosa 0.6.2 filters.mel(sr, n_fft, n_mels, fmin, fmax), htk=False, norm=1."""
    fmax = float(sr) / 2 if fmax is None else fmax
    bins = np.linspace(0, float(sr) / 2, 1 + n_fft // 2)
    edges = _mel_to_hz(np.linspace(_hz_to_mel(fmin)[0], _hz_to_mel(fmax)[0], n_mels + 2))
    lo, ce, hi = edges[:-2, None], edges[1:-1, None], edges[2:, None]
    rise = (bins[None, :] - lo) / (ce - lo)
    fall = (hi - bins[None, :]) / (hi - ce)
    w = np.maximum(0.0, np.minimum(rise, fall))
    return w * (2.0 / (edges[2:] - edges[:-2]))[:, None]


class AudioProcessor:
    def __init__(self, sample_rate=None, num_mels=None, min_level_db=None, frame_shift_ms=None,
                 frame_length_ms=None, ref_level_db=None, num_freq=None, power=None, preemphasis=None,
                 signal_norm=None, symmetric_norm=None, max_norm=None, mel_fmin=None, mel_fmax=None,
                 clip_norm=True, griffin_lim_iters=None, do_trim_silence=False, **kwargs):
        self.sample_rate = sample_rate
        self.num_mels = num_mels
        self.min_level_db = min_level_db
        self.frame_shift_ms = frame_shift_ms
        self.frame_length_ms = frame_length_ms
        self.ref_level_db = ref_level_db
        self.num_freq = num_freq
        self.power = power
        self.preemphasis = preemphasis
        self.griffin_lim_iters = griffin_lim_iters
        self.signal_norm = signal_norm
        self.symmetric_norm = symmetric_norm
        self.mel_fmin = 0 if mel_fmin is None else mel_fmin
        self.mel_fmax = mel_fmax
        self.max_norm = 1.0 if max_norm is None else float(max_norm)
        self.clip_norm = clip_norm
        self.do_trim_silence = do_trim_silence
        self.n_fft, self.hop_length, self.win_length = self._stft_parameters()
        self._gl = None
        self._mel_basis_set = False

    def _stft_parameters(self):  # utils/audio.py:114-119
        n_fft = (self.num_freq - 1) * 2
        hop_length = int(self.frame_shift_ms / 1000.0 * self.sample_rate)
        win_length = int(self.frame_length_ms / 1000.0 * self.sample_rate)
        return n_fft, hop_length, win_length

    def _build_mel_basis(self):  # utils/audio.py:68-77
        if self.mel_fmax is not None:
            assert self.mel_fmax <= self.sample_rate // 2
        return mel_basis(self.sample_rate, self.n_fft, self.num_mels, self.mel_fmin, self.mel_fmax)

    # ---------------------------------------------------------------- host helpers (not hot)
    def _denormalize(self, S):  # utils/audio.py:96-112
        if not self.signal_norm:
            return S
        if self.symmetric_norm:
            if self.clip_norm:
                S = np.clip(S, -self.max_norm, self.max_norm)
            return ((S + self.max_norm) * -self.min_level_db / (2 * self.max_norm)) + self.min_level_db
        if self.clip_norm:
            S = np.clip(S, 0, self.max_norm)
        return (S * -self.min_level_db / self.max_norm) + self.min_level_db

    def _db_to_amp(self, x):  # utils/audio.py:125-126
        return np.power(10.0, x * 0.05)

    def apply_inv_preemphasis(self, x):  # utils/audio.py:133-136
        if self.preemphasis == 0:
            raise RuntimeError(" !! Preemphasis is applied with factor 0.0. ")
        return scipy.signal.lfilter([1], [1, -self.preemphasis], x)

    def find_endpoint(self, wav, threshold_db=-40, min_silence_sec=0.8):  # utils/audio.py:203-210
        window_length = int(self.sample_rate * min_silence_sec)
        hop_length = int(window_length / 4)
        threshold = self._db_to_amp(threshold_db)
        for x in range(hop_length, len(wav) - window_length, hop_length):
            if np.max(wav[x:x + window_length]) < threshold:
                return x + hop_length
        return len(wav)

    def save_wav(self, wav, path):  # utils/audio.py:56-58
        wav_norm = np.asarray(wav) * (32767 / max(0.01, np.max(np.abs(wav))))
        scipy.io.wavfile.write(path, self.sample_rate, wav_norm.astype(np.int16))

    # ---------------------------------------------------------------- GPU Griffin-Lim
    def _handle(self):
        if self._gl is None:
            lib = _native.lib()
            cfg = _native.AudioConfig(
                n_fft=self.n_fft, hop_length=self.hop_length, win_length=self.win_length,
                num_mels=self.num_mels, min_level_db=self.min_level_db, ref_level_db=self.ref_level_db,
                power=self.power, max_norm=self.max_norm, preemphasis=float(self.preemphasis),
                signal_norm=int(bool(self.signal_norm)), symmetric_norm=int(bool(self.symmetric_norm)),
                clip_norm=int(bool(self.clip_norm)))
            pinv = np.ascontiguousarray(np.linalg.pinv(self._build_mel_basis()), dtype=np.float64)
            h = ctypes.c_void_p()
            _native.check(lib.tts_gl_create(ctypes.byref(cfg), pinv.ctypes.data_as(ctypes.c_void_p),
                                            _native.stream_handle(), ctypes.byref(h)), "tts_gl_create")
            self._gl = (lib, h)
        return self._gl

    def __del__(self):
        try:
            if self._gl is not None:
                self._gl[0].tts_gl_destroy(self._gl[1])
        except Exception:
            pass

    def griffin_lim_batch(self, spec, frames, mode=_native.TTS_GL_FROM_MEL, phase_u=None, seed=0, iters=None):
        """spec: CUDA fp32 [B, Fmax, n] (frame-major); frames: list of F_b.  Returns CUDA fp64
        [B, hop*(Fmax-1)]; sentence b's waveform is the first hop*(F_b-1) samples."""
        lib, h = self._handle()
        iters = self.griffin_lim_iters if iters is None else iters
        spec = spec.float().contiguous()
        B, Fmax = spec.shape[0], spec.shape[1]
        wav = torch.zeros(B, self.hop_length * (Fmax - 1), dtype=torch.float64, device=spec.device)
        pu = None
        if phase_u is not None:
            pu = torch.as_tensor(phase_u, dtype=torch.float64).to(spec.device).contiguous()
        _native.check(lib.tts_gl_run(h, mode, ctypes.c_void_p(spec.data_ptr()), _native.i32_array(frames), B, Fmax,
                                     ctypes.c_void_p(pu.data_ptr()) if pu is not None else None, int(seed), int(iters),
                                     ctypes.c_void_p(wav.data_ptr()), _native.stream_handle()), "tts_gl_run")
        return wav

    # ---------------------------------------------------------------- numpy-stream phases (device)
    @contextlib.contextmanager
    def numpy_phases(self):
        """Within the block, every Griffin-Lim run on this processor's handle with no explicit
        phase_u (griffin_lim_batch, and the one-call tts_synth_run of a model using it) draws its
        initial phases from numpy's global generator ON THE DEVICE: bitwise np.random.rand(1025, F_b)
        per sentence in batch order (utils/audio.py:183), without the host draw or its upload
        (tts_gl_set_phase_state, phase_mt.hip).  On exit numpy's global state is where the same
        draws would have left it."""
        lib, h = self._handle()
        st = np.random.get_state()
        if st[0] != "MT19937":
            raise RuntimeError("numpy's global generator is not the legacy MT19937")
        key = np.ascontiguousarray(st[1], dtype=np.uint32)
        _native.check(lib.tts_gl_set_phase_state(h, key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), int(st[2])),
                      "tts_gl_set_phase_state")
        try:
            yield self
            out = np.empty(624, np.uint32)
            pos = ctypes.c_int()
            _native.check(lib.tts_gl_get_phase_state(h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                                     ctypes.byref(pos)), "tts_gl_get_phase_state")
            np.random.set_state(("MT19937", out, pos.value, st[3], st[4]))
        finally:
            lib.tts_gl_set_phase_state(h, None, 0)

    def draw_phases(self, frames, Fmax=None):
        """The initial phases numpy_phases() gives a batch of these frame counts, as a CUDA fp64
        [B, 1025, Fmax] tensor (advances the armed state; zero past each sentence's frames)."""
        lib, h = self._handle()
        Fmax = max(frames) if Fmax is None else Fmax
        out = torch.zeros(len(frames), self.n_fft // 2 + 1, Fmax, dtype=torch.float64, device="cuda")
        _native.check(lib.tts_gl_draw_phases(h, _native.i32_array(frames), len(frames), Fmax,
                                             ctypes.c_void_p(out.data_ptr()), _native.stream_handle()),
                      "tts_gl_draw_phases")
        return out

    def pcm16_join(self, wav, lens, gap=0, peak=None):
        """Synthesizer.tts's join + save_wav's conversion on the device (tts_gl_save_pcm16): the
        first lens[b] samples of each row of the CUDA fp64 [B, pitch] ``wav``, each followed by
        ``gap`` zeros, times 32767 / max(0.01, peak) truncated to int16 (peak None: max |y| of the
        request).  Returns the int16 samples as a numpy array, bytes equal to numpy's."""
        lib, h = self._handle()
        wav = wav if wav.dim() == 2 else wav.view(1, -1)
        assert wav.dtype == torch.float64 and wav.is_cuda and wav.stride(1) == 1
        n = np.ascontiguousarray([int(x) for x in lens], dtype=np.int64)
        total = int(n.sum()) + gap * len(n)
        out = torch.empty(max(total, 1), dtype=torch.int16, device=wav.device)
        _native.check(lib.tts_gl_save_pcm16(h, ctypes.c_void_p(wav.data_ptr()), wav.stride(0),
                                            n.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), len(n), int(gap),
                                            -1.0 if peak is None else float(peak), ctypes.c_void_p(out.data_ptr()),
                                            _native.stream_handle()), "tts_gl_save_pcm16")
        return out[:total].cpu().numpy()

    def inv_mel_spectrogram_batch(self, mel, frames, seed=0, phase_u=None):
        return self.griffin_lim_batch(mel, frames, _native.TTS_GL_FROM_MEL, phase_u, seed)

    def last_gl_timing(self):
        lib, h = self._handle()
        ms, n = ctypes.c_float(), ctypes.c_int()
        lib.tts_gl_last_timing(h, ctypes.byref(ms), ctypes.byref(n))
        return dict(gl_loop_ms=ms.value, gl_iterations=n.value)

    def last_gl_path(self):
        """Iteration loop of the last run: "persistent", "fused" or "unfused" (tts_gl_last_path)."""
        lib, h = self._handle()
        p = ctypes.c_int()
        _native.check(lib.tts_gl_last_path(h, ctypes.byref(p)), "tts_gl_last_path")
        return _native.GL_PATHS[p.value]

    def profile_gl_kernels(self, reps=20):
        """Mean duration (ms) of the GL iteration and overlap-add kernels for the last batch."""
        lib, h = self._handle()
        n = len(_native.GL_KERNELS)
        ms = (ctypes.c_float * n)()
        _native.check(lib.tts_gl_profile(h, int(reps), ms, n), "tts_gl_profile")
        return dict(zip(_native.GL_KERNELS, [float(v) for v in ms]))

    # ---------------------------------------------------------------- mel analysis (GST style wavs)
    def melspectrogram_batch(self, wav, N):
        """wav: CUDA float64 [B, Nmax]; N: samples per sentence.  Returns (CUDA float32
        [B, Fmax, num_mels] frame-major, frames per sentence = 1 + N // hop)."""
        lib, h = self._handle()
        if not self._mel_basis_set:
            basis = np.ascontiguousarray(self._build_mel_basis(), dtype=np.float64)
            _native.check(lib.tts_gl_set_mel_basis(h, basis.ctypes.data_as(ctypes.c_void_p)), "tts_gl_set_mel_basis")
            self._mel_basis_set = True
        wav = wav.to(torch.float64).contiguous()
        B, Nmax = wav.shape
        F = [1 + int(n) // self.hop_length for n in N]
        mel = torch.empty(B, max(F), self.num_mels, device=wav.device)
        _native.check(lib.tts_gl_melspectrogram(h, ctypes.c_void_p(wav.data_ptr()), _native.i32_array(N), B, Nmax,
                                                ctypes.c_void_p(mel.data_ptr()), max(F), _native.stream_handle()),
                      "tts_gl_melspectrogram")
        return mel, F

    def melspectrogram(self, y):  # utils/audio.py:146-152 -> ndarray [num_mels, frames]
        self._handle()  # raises without a GPU / library: no CPU fallback
        y = np.asarray(y, dtype=np.float64)
        mel, F = self.melspectrogram_batch(torch.from_numpy(y).cuda()[None], [len(y)])
        return mel[0, :F[0]].T.double().cpu().numpy()

    def trim_silence(self, wav):
        """utils/audio.py:212-217 on the host: drop 0.1 s margins, then librosa 0.6.2
        effects.trim(top_db=40, frame_length=1024, hop_length=256) restated (rms of centre-padded
        frames, power_to_db against the max, keep frames above -top_db)."""
        margin = int(self.sample_rate * 0.1)
        wav = wav[margin:-margin]
        frame_length, hop_length, top_db = 1024, 256, 40
        yp = np.pad(wav, frame_length // 2, mode="reflect")
        n_frames = 1 + (len(yp) - frame_length) // hop_length
        idx = np.arange(frame_length)[:, None] + hop_length * np.arange(n_frames)[None, :]
        mse = np.sqrt(np.mean(np.abs(yp[idx]) ** 2, axis=0)) ** 2
        db = 10.0 * np.log10(np.maximum(1e-10, mse)) - 10.0 * np.log10(np.maximum(1e-10, mse.max()))
        nz = np.flatnonzero(db > -top_db)
        if nz.size == 0:
            return wav[0:0]
        return wav[int(nz[0]) * hop_length:min(len(wav), (int(nz[-1]) + 1) * hop_length)]

    def load_wav(self, filename, sr=None):
        """utils/audio.py:235-246 with soundfile's float64 conversion (PCM / 2**(bits-1))."""
        file_sr, x = scipy.io.wavfile.read(filename)
        if x.dtype == np.int16:
            x = x / 32768.0
        elif x.dtype == np.int32:
            x = x / 2147483648.0
        elif x.dtype == np.uint8:
            x = (x.astype(np.float64) - 128.0) / 128.0
        else:
            x = x.astype(np.float64)
        if self.do_trim_silence:
            x = self.trim_silence(x)
        assert self.sample_rate == file_sr, "%s vs %s" % (self.sample_rate, file_sr)
        return x

    def _single(self, spec_nT, mode):
        self._handle()  # raises without a GPU / library: no CPU fallback
        spec_nT = np.asarray(spec_nT, dtype=np.float32)
        T = spec_nT.shape[1]
        spec = torch.from_numpy(np.ascontiguousarray(spec_nT.T)).cuda()[None]
        # utils/audio.py:183: np.random.rand(1025, T) from numpy's global generator (unseeded unless
        # the caller seeds it), continued on the device
        with self.numpy_phases():
            wav = self.griffin_lim_batch(spec, [T], mode)
        return wav[0].cpu().numpy()

    def inv_mel_spectrogram(self, mel_spectrogram):  # utils/audio.py:164-172
        return self._single(mel_spectrogram, _native.TTS_GL_FROM_MEL)

    def inv_spectrogram(self, spectrogram):  # utils/audio.py:154-162
        return self._single(spectrogram, _native.TTS_GL_FROM_LINEAR)


def wav_bytes(ap: AudioProcessor, wav) -> _io.BytesIO:
    out = _io.BytesIO()
    ap.save_wav(np.asarray(wav), out)
    return out
