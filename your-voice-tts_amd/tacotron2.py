"""Drop-in for the reference ``Tacotron2`` (models/tacotron2.py:11-100) on MI355X.

Same constructor arguments, same ``state_dict`` keys and shapes (so reference checkpoints load
with ``load_state_dict(cp['model'])``), same ``inference(text, speaker_ids)`` return tuple
``(mel [B,T,80], mel_post [B,T,80], align [B,T,L], stop [B,T,1])``.

Where the compute runs:
  * decoder loop (``Decoder.inference``, layers/tacotron2.py:249-285): libtts_hip
    ``tts_decoder_run`` — HIP kernels, hipGraph-replayed steps;
  * Postnet + residual (layers/tacotron2.py:30-45, models/tacotron2.py:69-70): libtts_hip
    ``tts_postnet_run`` — fp32 MFMA implicit-GEMM convolutions;
  * embedding + encoder (layers/tacotron2.py:78-83): libtts_hip ``tts_encoder_run`` — the
    embedding gather fused into the first MFMA conv, BN folded, persistent BiLSTM.
There is no CPU path: without a GPU or without libtts_hip.so, ``inference`` raises.

Batches: the reference decoder is batch-1 (its stop rule reads item 0,
layers/tacotron2.py:268).  Here every sentence of a batch gets exactly the outputs it would get
alone; ``inference_batch`` takes ragged id lists, ``inference`` a [B, L] tensor.
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict

import numpy as np
import torch

from . import _native, weights


def _speaker_array(speaker_ids, B):
    """speaker ids as B int32 values: one id broadcasts to the batch (the reference's
    ``embedding(speaker_ids).unsqueeze(1)`` add, models/tacotron2.py:91-100), otherwise exactly one
    per sentence — the library reads B values, so a mismatch is rejected here, as torch's broadcast
    add would reject it."""
    spk = np.asarray(torch.as_tensor(speaker_ids).view(-1).cpu().numpy(), dtype=np.int32)
    if spk.size == 1 and B > 1:
        spk = np.repeat(spk, B)
    if spk.size != B:
        raise ValueError(f"speaker_ids has {spk.size} entries for a batch of {B}")
    return np.ascontiguousarray(spk)


class _DecoderAttrs:
    """Mutable attributes callers set on ``model.decoder`` (e.g. server/synthesizer.py:66)."""

    def __init__(self, r):
        self.max_decoder_steps = 1000  # layers/tacotron2.py:109
        self.r = r


class Tacotron2:
    def __init__(self, num_chars, num_speakers=0, r=1, attn_win=False, attn_norm="softmax",
                 prenet_type="original", prenet_dropout=True, forward_attn=False, trans_agent=False,
                 forward_attn_mask=False, location_attn=True, separate_stopnet=True,
                 max_batch=64, max_len=256, seed=0):
        if prenet_type not in ("original", "bn"):
            # common_layers.py:66-75 builds no layers for any other value (its forward then fails)
            raise ValueError(f"Unknown prenet_type {prenet_type!r}: expected 'original' or 'bn'")
        self.prenet_type = prenet_type
        if attn_norm not in ("softmax", "sigmoid"):
            raise RuntimeError("Unknown value for attention norm type")
        self.num_chars = num_chars
        self.num_speakers = num_speakers
        self.n_mel_channels = 80
        self.n_frames_per_step = r
        self.flags = dict(r=r, attn_norm=attn_norm, forward_attn=bool(forward_attn),
                          trans_agent=bool(trans_agent), forward_attn_mask=bool(forward_attn_mask),
                          location_attn=bool(location_attn), attn_win=bool(attn_win))
        self.separate_stopnet = separate_stopnet  # training-only flag (stopnet input detach)
        self.decoder = _DecoderAttrs(r)
        self.max_batch = max_batch
        self.max_len = max_len
        self.training = False
        self.device = torch.device("cpu")
        # prenet_type "bn": LinearBN layers (common_layers.py:28-52), folded into the prenet weights
        # and biases when the decoder handle is created (decoder_api.hip, fold_linear_bn)
        self._spec = weights.tacotron2_spec(num_chars, num_speakers, r, location_attn, trans_agent,
                                            prenet_bn=prenet_type == "bn")
        self._params = OrderedDict(
            (k, torch.from_numpy(v)) for k, v in weights.generate(self._spec, seed).items())
        self._native = None  # (decoder handle, postnet handle, key)
        self._synth = None  # (tts_synth handle, key, AudioProcessor)
        self._wav_buf = None
        self._enc_state = None  # inference_truncated: encoder BiLSTM state [4, 1, 256] (h_f, h_b, c_f, c_b)
        self._trunc_started = False  # inference_truncated: decoder states carried on the native handle
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
            raise RuntimeError(f"Error(s) in loading state_dict for Tacotron2: missing {missing}, "
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
        return [v for k, v in self._params.items() if v.is_floating_point()]

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
        self._lstm = None
        self._enc_state = None
        self._trunc_started = False
        if self._synth is not None:
            _native.load_library().tts_synth_destroy(self._synth[0])
            self._synth = None
        if self._native is not None:
            lib = _native.load_library()
            lib.tts_decoder_destroy(self._native[0])
            lib.tts_postnet_destroy(self._native[1])
            lib.tts_encoder_destroy(self._native[3])
            self._native = None

    def __del__(self):
        try:
            self._drop_native()
        except Exception:
            pass

    # ------------------------------------------------------------------ native handles
    def _handles(self, Lmax, B, need_steps=0):
        lib = _native.lib()
        if self.device.type != "cuda":
            self.cuda()
        # the decoder's history holds max_steps + 21 steps (teacher forcing may need more)
        max_steps = max(int(self.decoder.max_decoder_steps), need_steps - 21)
        key = (max_steps, max(self.max_len, Lmax), max(self.max_batch, B))
        if self._native is not None and (self._native[2][0] != max_steps or self._native[2][1] < Lmax
                                         or self._native[2][2] < B):
            self._drop_native()
        if self._native is None:
            f = self.flags
            cfg = _native.DecoderConfig(r=f["r"], attn_norm=0 if f["attn_norm"] == "softmax" else 1,
                                        forward_attn=int(f["forward_attn"]), trans_agent=int(f["trans_agent"]),
                                        forward_attn_mask=int(f["forward_attn_mask"]),
                                        location_attn=int(f["location_attn"]), windowing=int(f["attn_win"]),
                                        max_batch=key[2], max_len=key[1], max_steps=max_steps)
            stream = _native.stream_handle()
            dec_w = {k: v.float().contiguous() for k, v in self._params.items() if k.startswith("decoder.")}
            arr, keep = _native.tensor_views(dec_w)
            h = ctypes.c_void_p()
            _native.check(lib.tts_decoder_create(ctypes.byref(cfg), arr, len(dec_w), stream, ctypes.byref(h)),
                          "tts_decoder_create")
            post_w = {k: v.float().contiguous() for k, v in self._params.items()
                      if k.startswith("postnet.") and v.is_floating_point()}
            arr2, keep2 = _native.tensor_views(post_w)
            p = ctypes.c_void_p()
            _native.check(lib.tts_postnet_create(arr2, len(post_w), 80, stream, ctypes.byref(p)), "tts_postnet_create")
            enc_w = {k: v.float().contiguous() for k, v in self._params.items()
                     if (k.startswith("encoder.") or k in ("embedding.weight", "speaker_embedding.weight"))
                     and v.is_floating_point()}
            arr3, keep3 = _native.tensor_views(enc_w)
            e = ctypes.c_void_p()
            _native.check(lib.tts_encoder_create(arr3, len(enc_w), key[2], key[1], stream, ctypes.byref(e)),
                          "tts_encoder_create")
            self._native = (h, p, key, e)
        return lib, self._native[0], self._native[1]

    # ------------------------------------------------------------------ encoder
    @torch.no_grad()
    def encode(self, ids: torch.Tensor, lens, speaker_ids=None):
        """Embedding + Encoder.inference (models/tacotron2.py:63-66, layers/tacotron2.py:78-83)
        on a padded batch through libtts_hip ``tts_encoder_run``; every sentence is encoded at its
        own length (zero padding past it), as the reference does running it alone."""
        p = self._params
        B, Lmax = ids.shape
        lib, _, _ = self._handles(Lmax, B)
        ids32 = ids.to(self.device, dtype=torch.int32).contiguous()
        out = torch.empty(B, Lmax, 512, device=self.device)
        _native.check(lib.tts_encoder_run(self._native[3], ctypes.c_void_p(ids32.data_ptr()), _native.i32_array(lens),
                                          B, Lmax, ctypes.c_void_p(out.data_ptr()), _native.stream_handle()),
                      "tts_encoder_run")
        if speaker_ids is not None and "speaker_embedding.weight" in p:
            self._add_speakers(lib, out, lens, speaker_ids)
        return out

    def _add_speakers(self, lib, enc, lens, speaker_ids):
        """models/tacotron2.py:91-100 on the device (tts_encoder_add_speakers), in place."""
        B, Lmax = enc.shape[0], enc.shape[1]
        spk = _speaker_array(speaker_ids, B)
        _native.check(lib.tts_encoder_add_speakers(self._native[3], ctypes.c_void_p(enc.data_ptr()),
                                                   _native.i32_array(lens), _native.i32_array(spk), B, Lmax,
                                                   _native.stream_handle()), "tts_encoder_add_speakers")

    # ------------------------------------------------------------------ inference
    @torch.no_grad()
    def inference_batch(self, ids_list, speaker_ids=None, enc=None, lens=None, _continue=False):
        """Ragged batch: ids_list = list of 1-D id sequences.  Returns a dict of padded CUDA
        tensors (mel, mel_post [B,T,80]; align [B,Tsteps,L]; stop [B,Tsteps]) plus per-sentence
        ``frames`` (n_steps*r) and ``steps``."""
        _native.lib()  # raises without a GPU / library: no CPU fallback
        if enc is None:
            lens = [len(x) for x in ids_list]
            B, Lmax = len(lens), max(lens)
            ids = torch.zeros(B, Lmax, dtype=torch.long)
            for b, x in enumerate(ids_list):
                ids[b, :lens[b]] = torch.as_tensor(np.asarray(x), dtype=torch.long)
            if self.device.type != "cuda":
                self.cuda()
            enc = self.encode(ids.to(self.device), lens, speaker_ids)
        else:
            B, Lmax = enc.shape[0], enc.shape[1]
            lens = list(lens) if lens is not None else [Lmax] * B
        if min(lens) < 2:
            raise ValueError("encoder length must be >= 2 (the reference's forward-attention mask "
                             "indexes alpha[n-2], common_layers.py:213)")
        lib, hdec, hpost = self._handles(Lmax, B)
        r = self.n_frames_per_step
        max_steps = int(self.decoder.max_decoder_steps)
        cap = max_steps + 21
        dev = self.device
        enc = enc.float().contiguous()
        mel = torch.zeros(B, cap * r, 80, device=dev)
        stop = torch.zeros(B, cap, device=dev)
        align = torch.zeros(B, cap, Lmax, device=dev)
        n_steps = (ctypes.c_int32 * B)()
        stream = _native.stream_handle()
        run = lib.tts_decoder_run_continue if _continue else lib.tts_decoder_run
        _native.check(run(hdec, ctypes.c_void_p(enc.data_ptr()), _native.i32_array(lens), B, Lmax,
                          max_steps, cap, ctypes.c_void_p(mel.data_ptr()),
                          ctypes.c_void_p(stop.data_ptr()), ctypes.c_void_p(align.data_ptr()),
                          n_steps, stream), "tts_decoder_run")
        self._dec_enc = enc  # a batch-1 run reads it in place; profile_step_kernels re-reads it
        steps = [int(n_steps[b]) for b in range(B)]
        for s in steps:
            if s >= max_steps:
                print("   | > Decoder stopped with 'max_decoder_steps")  # layers/tacotron2.py:276
                break
        frames = [s * r for s in steps]
        mel_post = torch.zeros_like(mel)
        _native.check(lib.tts_postnet_run(hpost, ctypes.c_void_p(mel.data_ptr()), _native.i32_array(frames), B,
                                          cap * r, ctypes.c_void_p(mel_post.data_ptr()), stream), "tts_postnet_run")
        T, S = max(frames), max(steps)
        self.last_timing = self._path_timing(lib, hdec)
        self.last_lengths = frames
        return dict(mel=mel[:, :T], mel_post=mel_post[:, :T], align=align[:, :S], stop=stop[:, :S],
                    frames=frames, steps=steps, lens=lens)

    @torch.no_grad()
    def decoder_forward(self, inputs, memories, mask=None):
        """Decoder.forward(inputs, memories, mask) (layers/tacotron2.py:227-247), eval mode, teacher
        forcing: inputs [B, L, 512] encoder outputs, memories [B, T, 80] teacher mels, mask [B, L]
        (True = valid position; None = every sentence spans L).  Step t decodes from the go frame or
        teacher frame group t-1, T/r steps, no stop rule.  Returns (mel [B, 80, T], stop logits
        [B, T/r], alignments [B, T/r, L]) like the reference; each sentence is decoded at its own
        length (padding never attended)."""
        _native.lib()
        inputs = torch.as_tensor(inputs).to(self.device if self.device.type == "cuda" else "cuda").float().contiguous()
        B, L = inputs.shape[0], inputs.shape[1]
        lens = [L] * B if mask is None else [int(x) for x in torch.as_tensor(mask).reshape(B, -1).sum(1)]
        if min(lens) < 2:
            raise ValueError("encoder length must be >= 2 (common_layers.py:213)")
        r = self.n_frames_per_step
        memories = torch.as_tensor(memories).to(inputs.device).float().contiguous()
        T = memories.shape[1]
        if memories.dim() != 3 or memories.shape[0] != B or memories.shape[2] != 80 or T % r or T < r:
            raise ValueError(f"memories must be [B, T, 80] with T a positive multiple of r={r}")
        steps = T // r
        lib, hdec, _ = self._handles(L, B, need_steps=steps)
        mel = torch.empty(B, steps, 80 * r, device=inputs.device)
        stop = torch.empty(B, steps, device=inputs.device)
        align = torch.empty(B, steps, L, device=inputs.device)
        _native.check(lib.tts_decoder_run_teacher(hdec, ctypes.c_void_p(inputs.data_ptr()), _native.i32_array(lens), B, L,
                                                  ctypes.c_void_p(memories.data_ptr()), T * 80, steps,
                                                  ctypes.c_void_p(mel.data_ptr()), ctypes.c_void_p(stop.data_ptr()),
                                                  ctypes.c_void_p(align.data_ptr()), _native.stream_handle()),
                      "tts_decoder_run_teacher")
        return mel.view(B, steps * r, 80).transpose(1, 2), stop, align

    @torch.no_grad()
    def forward(self, text, text_lengths, mel_specs=None, speaker_ids=None):
        """Tacotron2.forward (models/tacotron2.py:47-60) in eval mode (training is out of scope):
        embedding + encoder at each sentence's length, teacher-forced decoder on mel_specs
        [B, T, 80], Postnet + residual.  Returns (mel [B, T, 80], mel_post [B, T, 80],
        alignments [B, T/r, L], stop logits [B, T/r]).  The reference's own forward cannot run on
        torch >= 1.2 (`1 - mask` on a bool mask, common_layers.py:234); this is its intended result."""
        if mel_specs is None:
            raise ValueError("Tacotron2.forward needs mel_specs (teacher forcing)")
        text = torch.as_tensor(text)
        lens = [int(x) for x in torch.as_tensor(text_lengths).reshape(-1)]
        B, Lmax = text.shape[0], max(lens)
        if self.device.type != "cuda":
            self.cuda()
        enc = self.encode(text[:, :Lmax].to(self.device), lens, speaker_ids)
        mask = torch.arange(Lmax)[None, :] < torch.as_tensor(lens)[:, None]
        mel, stop, align = self.decoder_forward(enc, mel_specs, mask)
        mel = mel.transpose(1, 2).contiguous()  # [B, T, 80]
        T = mel.shape[1]
        lib, _, hpost = self._handles(Lmax, B, need_steps=T // self.n_frames_per_step)
        mel_post = torch.empty_like(mel)
        _native.check(lib.tts_postnet_run(hpost, ctypes.c_void_p(mel.data_ptr()), _native.i32_array([T] * B), B, T,
                                          ctypes.c_void_p(mel_post.data_ptr()), _native.stream_handle()),
                      "tts_postnet_run")
        return mel, mel_post, align, stop

    @torch.no_grad()
    def inference(self, text, speaker_ids=None):
        """models/tacotron2.py:62-73.  text: LongTensor [B, L] (all rows length L)."""
        text = torch.as_tensor(text)
        if text.dim() == 1:
            text = text.unsqueeze(0)
        out = self.inference_batch([row for row in text.cpu().numpy()], speaker_ids=speaker_ids)
        return out["mel"], out["mel_post"], out["align"], out["stop"].unsqueeze(-1)

    @torch.no_grad()
    def synthesize_native(self, ids_list, ap, seed=0, iters=None, sync=True, speaker_ids=None, out=None):
        """utils/synthesis.py:synthesis (model.inference, :50-57 -> ap.inv_mel_spectrogram, :69-77)
        for a ragged batch in ONE native call (tts_synth_run): encoder -> decoder -> postnet ->
        Griffin-Lim with device phases from ``seed``, bitwise what inference_batch followed by
        ap.griffin_lim_batch(mel_post, frames, seed=seed) returns, without the host round trips
        between the stages.  Returns (wav: CUDA fp64 [B, hop*(Fmax-1)], frames).

        sync=True waits for the run and raises on its completion status; sync=False returns once
        Griffin-Lim is enqueued (the next call overlaps it and raises a failure of this one; a
        failed run's waveform is NaN, never a plausible signal).  ``out``: a CUDA fp64 buffer of at
        least ``native_wav_capacity(ap, B)`` elements to write into instead of the model's own (which
        the next call reuses).  Inside ``ap.numpy_phases()`` the phases are numpy's stream, not
        ``seed``'s."""
        if speaker_ids is not None and "speaker_embedding.weight" not in self._params:
            speaker_ids = None  # (the reference adds no embedding without the table either)
        lens = [len(x) for x in ids_list]
        if min(lens) < 2:
            raise ValueError("encoder length must be >= 2 (common_layers.py:213)")
        B, Lmax = len(lens), max(lens)
        lib, hdec, hpost = self._handles(Lmax, B)
        _, hgl = ap._handle()
        key = (self._native[2], id(ap), hgl.value if hasattr(hgl, "value") else int(hgl))
        if self._synth is not None and self._synth[1] != key:
            lib.tts_synth_destroy(self._synth[0])
            self._synth = None
        if self._synth is None:
            hs = ctypes.c_void_p()
            _native.check(lib.tts_synth_create(self._native[3], hdec, hpost, hgl, self.n_frames_per_step, 80,
                                               ap.hop_length, ctypes.byref(hs)), "tts_synth_create")
            # hold ap: its GL handle must outlive the synth handle
            self._synth = (hs, key, ap)
        hs = self._synth[0]
        max_steps = int(self.decoder.max_decoder_steps)
        ids = np.zeros((B, Lmax), np.int32)
        for b, x in enumerate(ids_list):
            ids[b, :lens[b]] = np.asarray(x, dtype=np.int32)
        # the decoder may legally run max_steps + 20 steps (the elif cap of layers/tacotron2.py:271-277
        # is skipped once every stop flag is set): size for the decoder's own steps_cap
        cap = self.native_wav_capacity(ap, B)
        if out is not None:
            if out.dtype != torch.float64 or not out.is_cuda or not out.is_contiguous() or out.numel() < cap:
                raise ValueError(f"out must be a contiguous CUDA float64 buffer of >= {cap} elements")
            wav_buf = out
        else:
            if self._wav_buf is None or self._wav_buf.numel() < cap:
                self._wav_buf = torch.empty(cap, dtype=torch.float64, device=self.device)
            wav_buf = self._wav_buf
        frames = (ctypes.c_int32 * B)()
        iters = ap.griffin_lim_iters if iters is None else iters
        if speaker_ids is None:
            _native.check(lib.tts_synth_run(hs, ids.ctypes.data_as(_native.I32P), _native.i32_array(lens), B, Lmax,
                                            max_steps, int(iters), int(seed), ctypes.c_void_p(wav_buf.data_ptr()),
                                            cap, frames, _native.stream_handle()), "tts_synth_run")
        else:
            spk = _speaker_array(speaker_ids, B)
            _native.check(lib.tts_synth_run_speakers(hs, ids.ctypes.data_as(_native.I32P), _native.i32_array(lens),
                                                     _native.i32_array(spk), B, Lmax, max_steps, int(iters), int(seed),
                                                     ctypes.c_void_p(wav_buf.data_ptr()), cap, frames,
                                                     _native.stream_handle()), "tts_synth_run_speakers")
        frames = [int(f) for f in frames]
        if sync:
            _native.check(lib.tts_synth_sync(hs), "tts_synth_sync")
        self.last_timing = self._path_timing(lib, hdec)
        self.last_lengths = frames
        n = ap.hop_length * (max(frames) - 1)
        return wav_buf.view(-1)[:B * n].view(B, n), frames

    def native_wav_capacity(self, ap, B=1):
        """Waveform elements one synthesize_native call of B sentences may write: the decoder may
        legally run max_steps + 20 steps (the elif cap of layers/tacotron2.py:271-277 is skipped once
        every stop flag is set), so the buffer is sized for the decoder's own steps_cap."""
        return B * ap.hop_length * ((int(self.decoder.max_decoder_steps) + 21) * self.n_frames_per_step - 1)

    def resident_limits(self, Lmax=1):
        """(max sentences, max encoder length) the resident decoder serves on this handle now
        (tts_decoder_resident_limits; (0, 0): multi-launch only)."""
        lib, hdec, _ = self._handles(max(int(Lmax), 1), 1)
        mb, ml = ctypes.c_int(), ctypes.c_int()
        _native.check(lib.tts_decoder_resident_limits(hdec, ctypes.byref(mb), ctypes.byref(ml)),
                      "tts_decoder_resident_limits")
        return mb.value, ml.value

    def synth_sync(self):
        """Wait for the last synthesize_native call and raise if its Griffin-Lim failed
        (tts_synth_sync); a no-op before the first call."""
        if self._synth is not None:
            _native.check(_native.lib().tts_synth_sync(self._synth[0]), "tts_synth_sync")

    def _path_timing(self, lib, hdec):
        """Decoder loop time and the paths the last run took (resident decoder / encoder BiLSTM)."""
        ms, ns, res, enc = ctypes.c_float(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        lib.tts_decoder_last_timing(hdec, ctypes.byref(ms), ctypes.byref(ns))
        lib.tts_decoder_last_path(hdec, ctypes.byref(res))
        lib.tts_encoder_last_path(self._native[3], ctypes.byref(enc))
        return dict(decoder_loop_ms=ms.value, decoder_steps_run=ns.value, resident=bool(res.value),
                    resident_kind=int(res.value), encoder_resident=bool(enc.value), encoder_path=int(enc.value))

    RESIDENT_PHASES = ("att_early_wait_pre1", "prenet2_row", "wait_prenet2", "att_lstm_prenet", "att_cell_gather",
                       "query_dec_early", "wait_query", "energies_max", "weights_ctx_publish", "next_prefetch",
                       "wait_ctx", "dec_lstm_ctx", "dec_cell_gather", "fused_rows", "cand_energies", "weights_ctx")

    def profile_resident_phases(self):
        """Mean µs per decoder step of each phase of the resident batch-1 decoder (last sentence
        re-run with timers; measurement only): {"cu0": {...}, "attention_cu": {...}}."""
        lib, hdec, _ = self._handles(1, 1)
        n = 2 * len(self.RESIDENT_PHASES)
        us = (ctypes.c_float * n)()
        _native.check(lib.tts_decoder_resident_phases(hdec, us, n), "tts_decoder_resident_phases")
        k = len(self.RESIDENT_PHASES)
        return {"cu0": dict(zip(self.RESIDENT_PHASES, [float(v) for v in us[:k]])),
                "attention_cu": dict(zip(self.RESIDENT_PHASES, [float(v) for v in us[k:]]))}

    def profile_resident_trace(self):
        """Per-CU event trace of the last resident sentence, re-run with event stamps only
        (measurement only): int64 numpy [256 CU, 64 steps, 12 events] of wall-clock ticks (P1, B1,
        h_att published, B3, B4, h_dec published, B6, pre1 row published, query row published;
        attention CUs: A1, A2, context published; 0 = not reached)."""
        lib, hdec, _ = self._handles(1, 1)
        n = 256 * 64 * 12
        buf = (ctypes.c_longlong * n)()
        _native.check(lib.tts_decoder_resident_trace(hdec, buf, n), "tts_decoder_resident_trace")
        return np.frombuffer(buf, dtype=np.int64).reshape(256, 64, 12).copy()

    def profile_step_kernels(self, reps=50):
        """Mean duration (ms) of each decoder-step kernel, HIP events on its own stream, for the
        batch of the last inference call (measurement only)."""
        lib, hdec, _ = self._handles(1, 1)
        n = len(_native.DECODER_STEP_KERNELS)
        ms = (ctypes.c_float * n)()
        _native.check(lib.tts_decoder_profile(hdec, int(reps), ms, n), "tts_decoder_profile")
        return dict(zip(_native.DECODER_STEP_KERNELS, [float(v) for v in ms]))

    @torch.no_grad()
    def inference_truncated(self, text, speaker_ids=None):
        """models/tacotron2.py:75-89, continuous inference over consecutive calls (batch 1): the
        encoder BiLSTM state (layers/tacotron2.py:85-93) and the decoder's RNN states, context and
        memory (:287-328) carry over; attention and stop rule restart.  Returns the same tuple as
        ``inference``."""
        _native.lib()
        text = torch.as_tensor(text)
        if text.dim() == 1:
            text = text.unsqueeze(0)
        if text.shape[0] != 1:
            raise ValueError("inference_truncated is batch-1 (the reference keeps one state per module)")
        L = int(text.shape[1])
        lib, _, _ = self._handles(L, 1)
        if self.flags["forward_attn_mask"] and L < 2:
            raise ValueError("encoder length must be >= 2 with forward_attn_mask")
        ids32 = text.to(self.device, dtype=torch.int32).contiguous()
        enc = torch.empty(1, L, 512, device=self.device)
        state_out = torch.empty(4, 1, 256, device=self.device)
        st_in = self._enc_state
        _native.check(lib.tts_encoder_run_state(
            self._native[3], ctypes.c_void_p(ids32.data_ptr()), _native.i32_array([L]), 1, L,
            ctypes.c_void_p(st_in.data_ptr()) if st_in is not None else None, ctypes.c_void_p(state_out.data_ptr()),
            ctypes.c_void_p(enc.data_ptr()), _native.stream_handle()), "tts_encoder_run_state")
        self._enc_state = state_out
        if speaker_ids is not None and "speaker_embedding.weight" in self._params:
            self._add_speakers(lib, enc, [L], speaker_ids)
        out = self.inference_batch(None, enc=enc, lens=[L], _continue=self._trunc_started)
        self._trunc_started = True
        return out["mel"], out["mel_post"], out["align"], out["stop"].unsqueeze(-1)

    __call__ = inference
