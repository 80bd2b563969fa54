"""Drop-ins for the reference ``TacotronGST`` (models/tacotrongst.py:10-90) and ``Tacotron``
(models/tacotron.py:9-81) on MI355X.

Same constructor arguments, ``state_dict`` keys and shapes (reference checkpoints load with
``load_state_dict(cp['model'])``), same ``inference`` return tuple
``(mel_outputs [B,T*r,80], linear_outputs [B,T*r,1025], alignments [B,T,L], stop_tokens [B,T])``.

Everything runs in libtts_hip (``tts_tacotron_*``, tacotron_api.hip): embedding + Prenet + CBHG
encoder, speaker embedding, the GST reference encoder and style-token attention, the
autoregressive decoder (hipGraph-replayed GRU steps with on-device stop rule), PostCBHG and the
linear projection.  There is no CPU path: without a GPU or the library, ``inference`` raises.

Batches: the reference decoder only runs batch 1 (its stop rule calls ``.item()``,
layers/tacotron.py:465); here every sentence of a padded batch gets exactly the outputs it would
get alone.
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict

import numpy as np
import torch

from . import _native, weights


class _DecoderAttrs:
    """Mutable attributes callers set on ``model.decoder`` (e.g. server/synthesizer.py:66)."""

    def __init__(self, r):
        self.max_decoder_steps = 500  # layers/tacotron.py:278
        self.r = r


class TacotronGST:
    _gst = True

    def __init__(self, num_chars, num_speakers, r=5, linear_dim=1025, mel_dim=80, memory_size=5, attn_win=False,
                 attn_norm="sigmoid", prenet_type="original", prenet_dropout=True, forward_attn=False,
                 trans_agent=False, forward_attn_mask=False, location_attn=True, separate_stopnet=True,
                 max_batch=64, max_len=256, seed=0):
        if prenet_type not in ("original", "bn"):
            # common_layers.py:66-75 builds no layers for any other value (its forward then fails)
            raise ValueError(f"Unknown prenet_type {prenet_type!r}: expected 'original' or 'bn'")
        self.prenet_type = prenet_type
        if attn_norm not in ("softmax", "sigmoid"):
            raise RuntimeError("Unknown value for attention norm type")
        if linear_dim != 1025 or mel_dim != 80:
            raise NotImplementedError("the MI355X path is built for linear_dim=1025, mel_dim=80")
        self.r = r
        self.mel_dim = mel_dim
        self.linear_dim = linear_dim
        self.memory_size = memory_size if memory_size > 0 else r
        if self.memory_size != r:
            raise NotImplementedError("memory_size != r is not on the MI355X path (every config uses 5 = r)")
        self.num_chars = num_chars
        self.num_speakers = num_speakers
        self.flags = dict(r=r, attn_norm=attn_norm, forward_attn=bool(forward_attn), trans_agent=bool(trans_agent),
                          forward_attn_mask=bool(forward_attn_mask), location_attn=bool(location_attn),
                          attn_win=bool(attn_win))
        self.separate_stopnet = separate_stopnet  # training-only flag
        self.decoder = _DecoderAttrs(r)
        self.max_batch = max_batch
        self.max_len = max_len
        self.training = False
        self.device = torch.device("cpu")
        self._spec = weights.tacotron_gst_spec(num_chars, num_speakers, r, self.memory_size, location_attn,
                                               trans_agent, gst=self._gst, prenet_bn=prenet_type == "bn")
        self._params = OrderedDict((k, torch.from_numpy(v)) for k, v in weights.generate(self._spec, seed).items())
        self._native = None  # (handle, key)
        self.last_lengths = None
        self.last_timing = {}

    # ------------------------------------------------------------------ module-like surface
    def state_dict(self):
        return OrderedDict((k, v) for k, v in self._params.items())

    def load_state_dict(self, sd, strict=True):
        want = {k: tuple(s) for k, s, _ in self._spec}
        missing = [k for k in want if k not in sd]
        unexpected = [k for k in sd if k not in want]
        if strict and (missing or unexpected):
            raise RuntimeError(f"Error(s) in loading state_dict for {type(self).__name__}: missing {missing}, "
                               f"unexpected {unexpected}")
        for k in want:
            if k not in sd:
                continue
            v = sd[k]
            v = v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))
            if tuple(v.shape) != want[k]:
                raise RuntimeError(f"size mismatch for {k}: copying a param with shape {tuple(v.shape)}, "
                                   f"the shape in current model is {want[k]}")
            self._params[k] = v.detach().to(self.device, dtype=self._params[k].dtype).contiguous()
        self._drop_native()
        return self

    def parameters(self):
        return [v for v in self._params.values() if v.is_floating_point()]

    def eval(self):
        self.training = False
        return self

    def train(self, mode=True):
        if mode:
            raise NotImplementedError("training is out of scope for the MI355X synthesis path")
        return self.eval()

    def to(self, device):
        self.device = torch.device(device)
        self._params = OrderedDict((k, v.to(self.device)) for k, v in self._params.items())
        self._drop_native()
        return self

    def cuda(self):
        return self.to("cuda")

    def cpu(self):
        return self.to("cpu")

    def _drop_native(self):
        if self._native is not None:
            _native.load_library().tts_tacotron_destroy(self._native[0])
            self._native = None

    def __del__(self):
        try:
            self._drop_native()
        except Exception:
            pass

    # ------------------------------------------------------------------ native handle
    def _handle(self, Lmax, B):
        lib = _native.lib()
        if self.device.type != "cuda":
            self.cuda()
        max_steps = int(self.decoder.max_decoder_steps)
        key = (max_steps, max(self.max_len, Lmax), max(self.max_batch, B))
        if self._native is not None and (self._native[1][0] != max_steps or self._native[1][1] < Lmax
                                         or self._native[1][2] < B):
            self._drop_native()
        if self._native is None:
            f = self.flags
            cfg = _native.TacotronConfig(
                r=f["r"], memory_size=self.memory_size, attn_norm=0 if f["attn_norm"] == "softmax" else 1,
                forward_attn=int(f["forward_attn"]), trans_agent=int(f["trans_agent"]),
                forward_attn_mask=int(f["forward_attn_mask"]), location_attn=int(f["location_attn"]),
                windowing=int(f["attn_win"]), gst=int(self._gst), num_speakers=int(self.num_speakers),
                max_batch=key[2], max_len=key[1], max_steps=max_steps)
            w = {k: v.float().contiguous() for k, v in self._params.items() if v.is_floating_point()}
            arr, keep = _native.tensor_views(w)
            h = ctypes.c_void_p()
            _native.check(lib.tts_tacotron_create(ctypes.byref(cfg), arr, len(w), _native.stream_handle(),
                                                  ctypes.byref(h)), "tts_tacotron_create")
            self._native = (h, key)
        return lib, self._native[0]

    # ------------------------------------------------------------------ encoder
    @staticmethod
    def _per_sentence(x, B):
        if x is None:
            return None
        x = np.asarray(x.cpu() if torch.is_tensor(x) else x).reshape(-1)
        if len(x) == 1 and B > 1:
            x = np.repeat(x, B)  # expand() over the batch (models/tacotrongst.py:86-88)
        if len(x) != B:
            raise ValueError(f"expected {B} speaker ids, got {len(x)}")
        return x

    @torch.no_grad()
    def encode(self, ids: torch.Tensor, lens, speaker_ids=None, style_mel=None):
        """embedding -> Encoder -> + speaker embedding -> + GST(style_mel) (models/tacotrongst.py:65-73)
        for a padded batch; every sentence encoded at its own length, rows past it zero."""
        B, Lmax = ids.shape
        lib, h = self._handle(Lmax, B)
        ids32 = ids.to(self.device, dtype=torch.int32).contiguous()
        out = torch.empty(B, Lmax, 256, device=self.device)
        sid = self._per_sentence(speaker_ids, B) if self.num_speakers > 1 else None
        sm, Ts = None, 0
        if style_mel is not None:
            if not self._gst:
                raise TypeError("Tacotron.inference takes no style_mel (models/tacotron.py:59)")
            sm = torch.as_tensor(style_mel, dtype=torch.float32).to(self.device)
            if sm.dim() == 2:
                sm = sm[None]
            # ReferenceEncoder.forward views its input as [B, 1, -1, num_mel] (gst_layers.py:60), so
            # compute_style_mel's [1, 80, T] tensor is read as rows of 80 consecutive values
            if sm[0].numel() % 80:
                raise ValueError(f"style_mel of {sm[0].numel()} values per sentence is not a whole number of "
                                 f"80-value rows")
            sm = sm.contiguous().view(sm.shape[0], -1, 80)
            if sm.shape[0] == 1 and B > 1:
                sm = sm.expand(B, -1, -1)  # gst_outputs broadcast over the batch (:71-73)
            if sm.shape[0] != B:
                raise ValueError(f"style_mel batch {sm.shape[0]} != {B}")
            sm = sm.contiguous()
            Ts = sm.shape[1]
        _native.check(lib.tts_tacotron_encode(
            h, ctypes.c_void_p(ids32.data_ptr()), _native.i32_array(lens), B, Lmax,
            _native.i32_array(sid) if sid is not None else None,
            ctypes.c_void_p(sm.data_ptr()) if sm is not None else None, Ts,
            ctypes.c_void_p(out.data_ptr()), _native.stream_handle()), "tts_tacotron_encode")
        return out

    # ------------------------------------------------------------------ inference
    @torch.no_grad()
    def inference_batch(self, ids_list, speaker_ids=None, style_mel=None, enc=None, lens=None, postnet=True):
        """Ragged batch: ids_list = list of 1-D id sequences.  Returns a dict of padded CUDA tensors
        (mel [B,T*r,80], linear [B,T*r,1025], align [B,T,L], stop [B,T]) plus per-sentence
        ``frames`` (steps*r) and ``steps``."""
        _native.lib()  # raises without a GPU / library: no CPU fallback
        if enc is None:
            lens = [len(x) for x in ids_list]
            B, Lmax = len(lens), max(lens)
            ids = torch.zeros(B, Lmax, dtype=torch.long)
            for b, x in enumerate(ids_list):
                ids[b, :lens[b]] = torch.as_tensor(np.asarray(x), dtype=torch.long)
            if self.device.type != "cuda":
                self.cuda()
            enc = self.encode(ids.to(self.device), lens, speaker_ids, style_mel)
        else:
            B, Lmax = enc.shape[0], enc.shape[1]
            lens = list(lens) if lens is not None else [Lmax] * B
        if self.flags["forward_attn_mask"] and min(lens) < 2:
            raise ValueError("encoder length must be >= 2 with forward_attn_mask "
                             "(the mask indexes alpha[n-2], common_layers.py:213)")
        lib, h = self._handle(Lmax, B)
        r = self.r
        max_steps = int(self.decoder.max_decoder_steps)
        cap = max_steps + 1
        dev = self.device
        enc = enc.float().contiguous()
        mel = torch.zeros(B, cap * r, 80, device=dev)
        stop = torch.zeros(B, cap, device=dev)
        align = torch.zeros(B, cap, Lmax, device=dev)
        n_steps = (ctypes.c_int32 * B)()
        stream = _native.stream_handle()
        _native.check(lib.tts_tacotron_decode(h, ctypes.c_void_p(enc.data_ptr()), _native.i32_array(lens), B, Lmax,
                                              max_steps, cap, ctypes.c_void_p(mel.data_ptr()),
                                              ctypes.c_void_p(stop.data_ptr()), ctypes.c_void_p(align.data_ptr()),
                                              n_steps, stream), "tts_tacotron_decode")
        steps = [int(n_steps[b]) for b in range(B)]
        if any(s > max_steps for s in steps):
            print("   | > Decoder stopped with 'max_decoder_steps")  # layers/tacotron.py:468
        frames = [s * r for s in steps]
        T, S = max(frames), max(steps)
        out = dict(mel=mel[:, :T], align=align[:, :S], stop=stop[:, :S], frames=frames, steps=steps, lens=lens)
        if postnet:
            out["linear"] = self.postnet(out["mel"], frames)
        ms, ns = ctypes.c_float(), ctypes.c_int()
        lib.tts_tacotron_last_timing(h, ctypes.byref(ms), ctypes.byref(ns))
        res = ctypes.c_int()
        lib.tts_tacotron_last_path(h, ctypes.byref(res))
        self.last_timing = dict(decoder_loop_ms=ms.value, decoder_steps_run=ns.value, resident=bool(res.value))
        self.last_lengths = frames
        return out

    @torch.no_grad()
    def postnet(self, mel, frames):
        """PostCBHG + last_linear + sigmoid (models/tacotrongst.py:77-78) on [B, T, 80] frames."""
        lib, h = self._handle(1, mel.shape[0])
        mel = mel.float().contiguous()
        B, T = mel.shape[0], mel.shape[1]
        lin = torch.empty(B, T, self.linear_dim, device=self.device)
        _native.check(lib.tts_tacotron_postnet(h, ctypes.c_void_p(mel.data_ptr()), _native.i32_array(frames), B, T,
                                               ctypes.c_void_p(lin.data_ptr()), _native.stream_handle()),
                      "tts_tacotron_postnet")
        return lin

    @torch.no_grad()
    def inference(self, characters, speaker_ids=None, style_mel=None):
        """models/tacotrongst.py:64-79.  characters: LongTensor [B, L] (all rows length L)."""
        characters = torch.as_tensor(characters)
        if characters.dim() == 1:
            characters = characters.unsqueeze(0)
        out = self.inference_batch([row for row in characters.cpu().numpy()], speaker_ids=speaker_ids,
                                   style_mel=style_mel)
        return out["mel"], out["linear"], out["align"], out["stop"]

    def profile_step_kernels(self, reps=20):
        """Mean duration (ms) of each decoder-step kernel for the batch of the last inference call."""
        lib, h = self._handle(1, 1)
        n = len(_native.TACOTRON_STEP_KERNELS)
        ms = (ctypes.c_float * n)()
        _native.check(lib.tts_tacotron_profile(h, int(reps), ms, n), "tts_tacotron_profile")
        return dict(zip(_native.TACOTRON_STEP_KERNELS, [float(v) for v in ms]))

    RESIDENT_PHASES = ("wait_pre1", "pre2_gather", "att_gru_gather", "query_gather", "attention_partial",
                       "leader_sum", "ctx_gather", "proj_gather", "gru1_gather", "gru2_gather", "mel_gather",
                       "pre1_stop", "att_gru_compute", "gru1_compute", "gru2_compute", "mel_compute")

    def profile_resident_phases(self):
        """Mean µs per decoder step of each phase of the resident decoder (last batch re-run with
        timers; measurement only): {"cu0": {...}, "cu1": {...}} (cu0 = an attention leader)."""
        lib, h = self._handle(1, 1)
        k = len(self.RESIDENT_PHASES)
        us = (ctypes.c_float * (2 * k))()
        _native.check(lib.tts_tacotron_resident_phases(h, us, 2 * k), "tts_tacotron_resident_phases")
        return {"cu0": dict(zip(self.RESIDENT_PHASES, [float(v) for v in us[:k]])),
                "cu1": dict(zip(self.RESIDENT_PHASES, [float(v) for v in us[k:]]))}

    __call__ = inference


class Tacotron(TacotronGST):
    """models/tacotron.py:9-81: TacotronGST without the GST block."""
    _gst = False

    def __init__(self, num_chars, num_speakers, r=5, linear_dim=1025, mel_dim=80, memory_size=5, attn_win=False,
                 attn_norm="sigmoid", prenet_type="original", prenet_dropout=True, forward_attn=False,
                 trans_agent=False, forward_attn_mask=False, location_attn=True, separate_stopnet=True, **kw):
        super().__init__(num_chars, num_speakers, r, linear_dim, mel_dim, memory_size, attn_win, attn_norm,
                         prenet_type, prenet_dropout, forward_attn, trans_agent, forward_attn_mask, location_attn,
                         separate_stopnet, **kw)

    @torch.no_grad()
    def inference(self, characters, speaker_ids=None):
        """models/tacotron.py:59-70."""
        return super().inference(characters, speaker_ids=speaker_ids, style_mel=None)

    __call__ = inference
