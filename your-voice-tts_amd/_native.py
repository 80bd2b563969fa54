"""ctypes binding of libtts_hip.so (C-ABI in include/tts_hip.h).

The library is loaded on first use.  If it is missing, fails to load, or no GPU is visible, the
caller gets a RuntimeError: the product path has no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TTS_HIP_LIB", os.path.join(_HERE, "libtts_hip.so"))

TTS_GL_FROM_MEL = 0
TTS_GL_FROM_LINEAR = 1
GL_PATHS = {0: "unfused", 1: "fused", 2: "persistent"}  # TTS_GL_PATH_* (include/tts_hip.h)
DECODER_STEP_KERNELS = ("prenet2", "att_lstm", "query", "attention", "dec_lstm", "mel_fused")
GL_KERNELS = ("gl_iter", "gl_ola")
TACOTRON_STEP_KERNELS = ("prenet2", "att_gru", "query", "attention", "proj", "dec_gru1", "dec_gru2", "mel",
                         "pre1_stop")

# every symbol include/tts_hip.h declares
EXPORTS = (
    "tts_encoder_create", "tts_encoder_destroy", "tts_encoder_run", "tts_encoder_run_state", "tts_encoder_last_path",
    "tts_encoder_add_speakers", "tts_synth_run_speakers",
    "tts_decoder_create", "tts_decoder_destroy", "tts_decoder_run", "tts_decoder_run_continue", "tts_decoder_run_teacher",
    "tts_decoder_last_timing", "tts_decoder_last_path", "tts_decoder_resident_limits", "tts_decoder_resident_phases", "tts_decoder_resident_trace",
    "tts_decoder_profile",
    "tts_postnet_create", "tts_postnet_destroy", "tts_postnet_run",
    "tts_gl_create", "tts_gl_destroy", "tts_gl_run", "tts_gl_last_timing", "tts_gl_last_path", "tts_gl_profile",
    "tts_gl_set_mel_basis", "tts_gl_melspectrogram", "tts_gl_set_phase_state", "tts_gl_get_phase_state",
    "tts_gl_draw_phases", "tts_gl_save_pcm16",
    "tts_synth_create", "tts_synth_destroy", "tts_synth_run", "tts_synth_sync",
    "tts_tacotron_create", "tts_tacotron_destroy", "tts_tacotron_encode", "tts_tacotron_decode",
    "tts_tacotron_postnet", "tts_tacotron_last_timing", "tts_tacotron_last_path", "tts_tacotron_resident_phases",
    "tts_tacotron_profile",
    "tts_last_error", "tts_version",
)


class TensorView(ctypes.Structure):
    _fields_ = [("key", ctypes.c_char_p), ("data", ctypes.c_void_p), ("numel", ctypes.c_int64)]


class DecoderConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "r", "attn_norm", "forward_attn", "trans_agent", "forward_attn_mask", "location_attn",
        "windowing", "max_batch", "max_len", "max_steps")]


class TacotronConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "r", "memory_size", "attn_norm", "forward_attn", "trans_agent", "forward_attn_mask", "location_attn",
        "windowing", "gst", "num_speakers", "max_batch", "max_len", "max_steps")]


class AudioConfig(ctypes.Structure):
    _fields_ = [("n_fft", ctypes.c_int), ("hop_length", ctypes.c_int), ("win_length", ctypes.c_int),
                ("num_mels", ctypes.c_int), ("min_level_db", ctypes.c_float),
                ("ref_level_db", ctypes.c_float), ("power", ctypes.c_float),
                ("max_norm", ctypes.c_float), ("preemphasis", ctypes.c_double),
                ("signal_norm", ctypes.c_int), ("symmetric_norm", ctypes.c_int), ("clip_norm", ctypes.c_int)]


_lib = None
_lock = threading.Lock()
P = ctypes.c_void_p
I32P = ctypes.POINTER(ctypes.c_int32)


def _declare(lib):
    vp = ctypes.c_void_p
    lib.tts_encoder_create.argtypes = [ctypes.POINTER(TensorView), ctypes.c_int, ctypes.c_int, ctypes.c_int, vp,
                                       ctypes.POINTER(vp)]
    lib.tts_encoder_destroy.argtypes = [vp]
    lib.tts_encoder_destroy.restype = None
    lib.tts_encoder_run.argtypes = [vp, vp, I32P, ctypes.c_int, ctypes.c_int, vp, vp]
    lib.tts_encoder_add_speakers.argtypes = [vp, vp, I32P, I32P, ctypes.c_int, ctypes.c_int, vp]
    lib.tts_decoder_create.argtypes = [ctypes.POINTER(DecoderConfig), ctypes.POINTER(TensorView), ctypes.c_int, vp,
                                       ctypes.POINTER(vp)]
    lib.tts_decoder_destroy.argtypes = [vp]
    lib.tts_decoder_destroy.restype = None
    lib.tts_decoder_run.argtypes = [vp, vp, I32P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, vp,
                                    I32P, vp]
    lib.tts_encoder_run_state.argtypes = [vp, vp, I32P, ctypes.c_int, ctypes.c_int, vp, vp, vp, vp]
    lib.tts_decoder_run_continue.argtypes = lib.tts_decoder_run.argtypes
    lib.tts_decoder_run_teacher.argtypes = [vp, vp, I32P, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int64, ctypes.c_int,
                                            vp, vp, vp, vp]
    lib.tts_decoder_last_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)]
    lib.tts_decoder_last_path.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
    lib.tts_decoder_resident_limits.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    lib.tts_encoder_last_path.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
    lib.tts_gl_last_path.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
    lib.tts_synth_sync.argtypes = [vp]
    lib.tts_decoder_resident_phases.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.c_int]
    lib.tts_decoder_resident_trace.argtypes = [vp, ctypes.POINTER(ctypes.c_longlong), ctypes.c_int64]
    lib.tts_postnet_create.argtypes = [ctypes.POINTER(TensorView), ctypes.c_int, ctypes.c_int, vp, ctypes.POINTER(vp)]
    lib.tts_postnet_destroy.argtypes = [vp]
    lib.tts_postnet_destroy.restype = None
    lib.tts_postnet_run.argtypes = [vp, vp, I32P, ctypes.c_int, ctypes.c_int, vp, vp]
    lib.tts_gl_create.argtypes = [ctypes.POINTER(AudioConfig), vp, vp, ctypes.POINTER(vp)]
    lib.tts_gl_destroy.argtypes = [vp]
    lib.tts_gl_destroy.restype = None
    lib.tts_gl_run.argtypes = [vp, ctypes.c_int, vp, I32P, ctypes.c_int, ctypes.c_int, vp, ctypes.c_uint64,
                               ctypes.c_int, vp, vp]
    lib.tts_gl_set_mel_basis.argtypes = [vp, vp]
    lib.tts_gl_melspectrogram.argtypes = [vp, vp, I32P, ctypes.c_int, ctypes.c_int64, vp, ctypes.c_int, vp]
    lib.tts_gl_last_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)]
    U32P = ctypes.POINTER(ctypes.c_uint32)
    lib.tts_gl_set_phase_state.argtypes = [vp, U32P, ctypes.c_int]
    lib.tts_gl_get_phase_state.argtypes = [vp, U32P, ctypes.POINTER(ctypes.c_int)]
    lib.tts_gl_draw_phases.argtypes = [vp, I32P, ctypes.c_int, ctypes.c_int, vp, vp]
    lib.tts_gl_save_pcm16.argtypes = [vp, vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64), ctypes.c_int, ctypes.c_int,
                                      ctypes.c_double, vp, vp]
    lib.tts_synth_create.argtypes = [vp, vp, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
    lib.tts_synth_destroy.argtypes = [vp]
    lib.tts_synth_destroy.restype = None
    lib.tts_synth_run.argtypes = [vp, I32P, I32P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_uint64, vp, ctypes.c_int64, I32P, vp]
    lib.tts_synth_run_speakers.argtypes = [vp, I32P, I32P, I32P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_uint64, vp, ctypes.c_int64, I32P, vp]
    FP = ctypes.POINTER(ctypes.c_float)
    lib.tts_decoder_profile.argtypes = [vp, ctypes.c_int, FP, ctypes.c_int]
    lib.tts_gl_profile.argtypes = [vp, ctypes.c_int, FP, ctypes.c_int]
    lib.tts_tacotron_create.argtypes = [ctypes.POINTER(TacotronConfig), ctypes.POINTER(TensorView), ctypes.c_int, vp,
                                        ctypes.POINTER(vp)]
    lib.tts_tacotron_destroy.argtypes = [vp]
    lib.tts_tacotron_destroy.restype = None
    lib.tts_tacotron_encode.argtypes = [vp, vp, I32P, ctypes.c_int, ctypes.c_int, I32P, vp, ctypes.c_int, vp, vp]
    lib.tts_tacotron_decode.argtypes = [vp, vp, I32P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp,
                                        vp, I32P, vp]
    lib.tts_tacotron_postnet.argtypes = [vp, vp, I32P, ctypes.c_int, ctypes.c_int, vp, vp]
    lib.tts_tacotron_last_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)]
    lib.tts_tacotron_last_path.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
    lib.tts_tacotron_resident_phases.argtypes = [vp, FP, ctypes.c_int]
    lib.tts_tacotron_profile.argtypes = [vp, ctypes.c_int, FP, ctypes.c_int]
    lib.tts_last_error.restype = ctypes.c_char_p
    lib.tts_version.restype = ctypes.c_char_p
    for name in EXPORTS:
        fn = getattr(lib, name)
        if name.endswith(("_create", "_run", "_timing", "_profile", "_encode", "_decode", "_postnet", "_state",
                          "_continue", "_basis", "_melspectrogram", "_path", "_sync", "_phases", "_teacher",
                          "_phase_state", "_pcm16", "_limits")):
            fn.restype = ctypes.c_int


def load_library(path: str = LIB_PATH):
    """Load (once) and return the ctypes handle.  torch is imported first so that the HIP
    runtime torch ships (SONAME libamdhip64.so.7) is the one the library binds to."""
    global _lib
    with _lock:
        if _lib is None:
            import torch  # noqa: F401  (HIP runtime first)
            if not os.path.exists(path):
                raise RuntimeError(f"libtts_hip.so not found at {path}: build it with "
                                   f"`make -C your-voice-tts_amd/csrc` (no CPU fallback exists)")
            lib = ctypes.CDLL(path)
            _declare(lib)
            _lib = lib
    return _lib


def lib():
    """Library handle for compute calls: requires a visible GPU."""
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("no GPU visible: the MI355X synthesis path has no CPU fallback")
    return load_library()


def check(status: int, what: str):
    if status != 0:
        msg = load_library().tts_last_error().decode(errors="replace")
        if "attention norm" in msg:
            raise RuntimeError("Unknown value for attention norm type")
        raise RuntimeError(f"{what} failed (status {status}): {msg}")


def stream_handle(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def tensor_views(tensors: dict):
    """Build a TensorView array over CUDA tensors; returns (array, keepalive)."""
    items = list(tensors.items())
    arr = (TensorView * len(items))()
    keep = []
    for i, (k, t) in enumerate(items):
        kb = k.encode()
        keep.append(kb)
        keep.append(t)
        arr[i].key = kb
        arr[i].data = t.data_ptr()
        arr[i].numel = t.numel()
    return arr, keep


def i32_array(values):
    vals = [int(v) for v in values]
    return (ctypes.c_int32 * len(vals))(*vals)
