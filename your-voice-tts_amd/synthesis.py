"""Callers of the synthesis path: ``synthesis`` (utils/synthesis.py:78-124), ``tts``
(synthesize.py:15-38) and ``Synthesizer`` (server/synthesizer.py:22-162), plus the batched
GPU-resident pipeline they share.

The text front-end (phonemizer/espeak, utils/text/) is outside the MI355X path and its
dependencies are not installed here: callers pass character/phoneme ids, or give
``Synthesizer`` an ``input_adapter`` (the reference builds one at server/synthesizer.py:51-54).
"""
from __future__ import annotations

import io
import os
import re
import time

import numpy as np
import torch

from . import _native
from .audio import AudioProcessor

# ------------------------------------------------------------------ sentence splitting
# server/synthesizer.py:12-17, 102-126 (regex pipeline restated)
_ALPHA = "([A-Za-z])"
_PREFIXES = "(Mr|St|Mrs|Ms|Dr)[.]"
_SUFFIXES = "(Inc|Ltd|Jr|Sr|Co)"
_STARTERS = r"(Mr|Mrs|Ms|Dr|He\s|She\s|It\s|They\s|Their\s|Our\s|We\s|But\s|However\s|That\s|This\s|Wherever)"
_ACRONYMS = "([A-Z][.][A-Z][.](?:[A-Z][.])?)"
_WEBSITES = "[.](com|net|org|io|gov)"


def split_into_sentences(text: str):
    t = " " + text + "  "
    t = t.replace("\n", " ")
    t = re.sub(_PREFIXES, "\\1<prd>", t)
    t = re.sub(_WEBSITES, "<prd>\\1", t)
    if "Ph.D" in t:
        t = t.replace("Ph.D.", "Ph<prd>D<prd>")
    t = re.sub(r"\s" + _ALPHA + "[.] ", " \\1<prd> ", t)
    t = re.sub(_ACRONYMS + " " + _STARTERS, "\\1<stop> \\2", t)
    t = re.sub(_ALPHA + "[.]" + _ALPHA + "[.]" + _ALPHA + "[.]", "\\1<prd>\\2<prd>\\3<prd>", t)
    t = re.sub(_ALPHA + "[.]" + _ALPHA + "[.]", "\\1<prd>\\2<prd>", t)
    t = re.sub(" " + _SUFFIXES + "[.] " + _STARTERS, " \\1<stop> \\2", t)
    t = re.sub(" " + _SUFFIXES + "[.]", " \\1<prd>", t)
    t = re.sub(" " + _ALPHA + "[.]", " \\1<prd>", t)
    if "”" in t:
        t = t.replace(".”", "”.")
    if '"' in t:
        t = t.replace('."', '".')
    if "!" in t:
        t = t.replace('!"', '"!')
    if "?" in t:
        t = t.replace('?"', '"?')
    t = t.replace(".", ".<stop>").replace("?", "?<stop>").replace("!", "!<stop>").replace("<prd>", ".")
    return [s.strip() for s in t.split("<stop>")[:-1]]


def wav_to_int16(wav):
    """save_wav's conversion (utils/audio.py:56-58): peak-normalise to 32767, truncate to int16."""
    wav = np.asarray(wav)
    return (wav * (32767 / max(0.01, np.max(np.abs(wav))))).astype(np.int16)


# ------------------------------------------------------------------ batched pipeline
# Requests of at most this many Tacotron2 sentences decode one sentence at a time on the resident
# batch-1 decoder instead of as one multi-launch batch (tools/dispatch_crossover.py,
# profiles/r05_dispatch_crossover.json: 3 sentences 102.6 vs 128.8 ms under the Synthesizer's
# mask-off 3000-step configuration, 8.5 vs 12.7 ms under synthesize.py's mask; from 4 on the batch
# wins).  Postnet per sentence, Griffin-Lim still one batch.  TTS_SERIAL_MAX overrides (0: off).
SERIAL_RESIDENT_MAX = int(os.environ.get("TTS_SERIAL_MAX", "3"))


def _decode(model, ids_list, speaker_ids=None):
    """Tacotron2 decode of a request: serial resident calls below the crossover, else one batch."""
    B = len(ids_list)
    if B == 1 or B > SERIAL_RESIDENT_MAX or max(len(x) for x in ids_list) > 256:
        out = model.inference_batch(ids_list, speaker_ids=speaker_ids)
        out["dispatch"] = "batch"
        return out
    from .tacotron2 import _speaker_array
    spk = None if speaker_ids is None else _speaker_array(speaker_ids, B)
    outs = []
    for b, x in enumerate(ids_list):
        outs.append(model.inference_batch([x], speaker_ids=None if spk is None else spk[b:b + 1]))
        if b == 0 and not model.last_timing.get("resident"):
            # no resident decoder on this handle: the rest as one batch is cheaper
            outs.append(model.inference_batch(ids_list[1:], speaker_ids=None if spk is None else spk[1:]))
            break
    frames = [f for o in outs for f in o["frames"]]
    steps = [n for o in outs for n in o["steps"]]
    T = max(frames)
    mel_post = torch.zeros(B, T, outs[0]["mel_post"].shape[2], device=outs[0]["mel_post"].device)
    b = 0
    for o in outs:
        for k in range(len(o["frames"])):
            mel_post[b, :o["frames"][k]] = o["mel_post"][k, :o["frames"][k]]
            b += 1
    return dict(mel_post=mel_post, frames=frames, steps=steps, dispatch="serial-resident")


@torch.no_grad()
def synthesize_batch(model, ap: AudioProcessor, ids_list, speaker_ids=None, seed=0, phase="device",
                     iters=None, keep_outputs=False, style_mel=None):
    """ids -> encoder -> HIP decoder -> HIP postnet -> HIP Griffin-Lim for a ragged batch.

    phase: "device" draws the initial GL phases on the GPU from ``seed``; "numpy" draws them
    sentence by sentence with np.random.rand(1025, T_b) in batch order, as the reference does
    when it synthesises the sentences one after another.  Returns (wavs: list of float64 numpy
    arrays, info dict)."""
    linear = hasattr(model, "linear_dim")  # Tacotron / TacotronGST: linear-spectrogram GL
    if linear:
        out = model.inference_batch(ids_list, speaker_ids=speaker_ids, style_mel=style_mel)
    else:  # (keep_outputs or not: the same dispatch, so a sharded rank decodes as the single process does)
        out = _decode(model, ids_list, speaker_ids)
    frames = out["frames"]
    mel_post = out["linear"] if linear else out["mel_post"]
    phase_u = None
    if phase == "numpy":
        Fmax = mel_post.shape[1]
        phase_u = np.zeros((len(frames), ap.n_fft // 2 + 1, Fmax))
        for b, T in enumerate(frames):
            phase_u[b, :, :T] = np.random.rand(ap.n_fft // 2 + 1, T)
    mode = _native.TTS_GL_FROM_LINEAR if linear else _native.TTS_GL_FROM_MEL
    wav = ap.griffin_lim_batch(mel_post, frames, mode=mode, phase_u=phase_u, seed=seed, iters=iters)
    lens = [ap.hop_length * (T - 1) for T in frames]
    info = dict(frames=frames, steps=out["steps"], samples=lens, decoder_dispatch=out.get("dispatch", "batch"),
                **model.last_timing, **ap.last_gl_timing())
    if keep_outputs:
        info.update(out)
        info["wav_dev"] = wav
    wav_h = wav.cpu().numpy()
    return [wav_h[b, :n] for b, n in enumerate(lens)], info


# ------------------------------------------------------------------ reference call sites
def text_to_seqvec(text, CONFIG):
    """utils/synthesis.py:11-25 (host): ids of a sentence.  Character configs go through
    text.text_to_sequence; phoneme configs need phonemizer/espeak (not installed) and raise."""
    from . import text as _text
    if CONFIG.get("use_phonemes", False):
        return _text.phoneme_to_sequence(text, [CONFIG.text_cleaner], CONFIG.phoneme_language,
                                         CONFIG.get("enable_eos_bos_chars", False))
    return _text.text_to_sequence(text, [CONFIG.text_cleaner])


def _ids_tensor(text, CONFIG):
    if isinstance(text, str):
        text = text_to_seqvec(text, CONFIG)
    return torch.as_tensor(np.asarray(text), dtype=torch.long).view(1, -1)


def compute_style_mel(style_wav, ap, use_cuda=True):
    """utils/synthesis.py:28-35: ``style_wav`` a wav path -> FloatTensor(ap.melspectrogram(
    ap.load_wav(path))).unsqueeze(0), i.e. [1, 80, frames] (the GST reads it with a view as rows of
    80 values, layers/gst_layers.py:60, exactly like the reference); or an already computed style
    mel tensor / array, passed through."""
    if isinstance(style_wav, (str, bytes, os.PathLike)):
        style = ap.melspectrogram(ap.load_wav(style_wav))  # [80, frames] float64 -> float32 below
    else:
        style = style_wav.cpu().numpy() if torch.is_tensor(style_wav) else np.asarray(style_wav)
    style = torch.as_tensor(np.asarray(style, dtype=np.float32))
    if style.dim() == 2:
        style = style[None]
    return style.cuda() if use_cuda else style


def run_model(model, inputs, CONFIG, truncated, speaker_id=None, style_mel=None):
    """utils/synthesis.py:38-49: GST with a style mel -> inference(style_mel=...); otherwise
    inference_truncated (continuous mode) or inference."""
    if CONFIG.model == "TacotronGST" and style_mel is not None:
        return model.inference(inputs, style_mel=style_mel, speaker_ids=speaker_id)
    if truncated:
        return model.inference_truncated(inputs, speaker_ids=speaker_id)
    return model.inference(inputs, speaker_ids=speaker_id)


def synthesis(model, text, CONFIG, use_cuda, ap, speaker_id=None, style_wav=None, truncated=False,
              enable_eos_bos_chars=False, trim_silence=False):
    """utils/synthesis.py:78-124: returns (wav, alignment [T,L], decoder_output [T*r,80],
    postnet_output [T*r,80] (Tacotron2) or [T*r,1025] (Tacotron / TacotronGST), stop_tokens) for
    both values of ``truncated`` (run_model picks inference / inference_truncated; parse_outputs and
    the Griffin-Lim tail are the same)."""
    style_mel = None
    if CONFIG.model == "TacotronGST" and style_wav is not None:
        style_mel = compute_style_mel(style_wav, ap, use_cuda)
    inputs = _ids_tensor(text, CONFIG)
    sid = None if speaker_id is None or speaker_id is False else torch.as_tensor([speaker_id])
    decoder_output, postnet_output, alignments, stop_tokens = run_model(model, inputs, CONFIG, truncated, sid,
                                                                        style_mel)
    postnet_output = postnet_output[0].cpu().numpy()  # parse_outputs (utils/synthesis.py:52-56)
    decoder_output = decoder_output[0].cpu().numpy()
    alignment = alignments[0].cpu().numpy()
    if CONFIG.model in ("Tacotron", "TacotronGST"):  # inv_spectrogram (utils/synthesis.py:63-68)
        wav = ap.inv_spectrogram(postnet_output.T)
    else:
        wav = ap.inv_mel_spectrogram(postnet_output.T)
    if trim_silence:
        # the reference's intent (utils/synthesis.py:59-60): cut at AudioProcessor.find_endpoint.
        # (Its parameter shadows the module function, so the reference itself raises TypeError here.)
        wav = wav[:ap.find_endpoint(wav)]
    return wav, alignment, decoder_output, postnet_output, stop_tokens


def tts(model, vocoder_model, C, VC, text, ap, use_cuda, batched_vocoder, figures=False):
    """synthesize.py:15-38 with the GL vocoder (WaveRNN is an external repo, not vendored)."""
    if vocoder_model is not None:
        raise NotImplementedError("WaveRNN vocoder is not part of the reference tree")
    t_1 = time.time()
    waveform, alignment, decoder_outputs, postnet_output, stop_tokens = synthesis(
        model, text, C, use_cuda, ap, None, None, False, C.enable_eos_bos_chars)
    print(" >  Run-time: {}".format(time.time() - t_1))
    return alignment, postnet_output, stop_tokens, waveform


class Synthesizer:
    """server/synthesizer.py:29-162.  Built like the reference, from the server config
    (``Synthesizer(config)`` with tts_path / tts_file / tts_config / use_cuda: ``load_tts`` reads
    the model config and checkpoint), or from parts: a built model, an AudioProcessor, the tts config
    and an input_adapter (sentence -> ids).  All sentences of a request are synthesised as one GPU
    batch instead of one after another."""

    def __init__(self, tts_model, ap=None, tts_config=None, input_adapter=None, seed=0):
        self.seed = seed
        self.wavernn = None
        if ap is None and tts_config is None and isinstance(tts_model, dict) and "tts_path" in tts_model:
            # server/synthesizer.py:30-38: Synthesizer(config)
            self.config = tts_model
            self.use_cuda = self.config.get("use_cuda", True)
            self.load_tts(self.config["tts_path"], self.config["tts_file"], self.config["tts_config"], self.use_cuda)
            if self.config.get("wavernn_lib_path"):
                raise NotImplementedError("WaveRNN (server/synthesizer.py:68-95) is an external repo, not part "
                                          "of the reference tree: leave wavernn_lib_path empty for Griffin-Lim")
            return
        self.tts_model = tts_model
        self.ap = ap
        self.tts_config = tts_config
        self.input_adapter = input_adapter
        self.tts_model.eval()
        self.tts_model.decoder.max_decoder_steps = 3000  # server/synthesizer.py:66

    def load_tts(self, model_path, model_file, model_config, use_cuda=True):
        """server/synthesizer.py:40-66: config -> AudioProcessor, the input adapter (phonemes or
        characters), setup_model, cp['model'] (weights-only load), eval, 3000-step decoder cap.
        The model always runs on the GPU (no CPU path), whatever use_cuda says."""
        from . import text as _text
        from .generic_utils import load_config
        from .synthesize import load_model
        tts_config = os.path.join(model_path, model_config)
        self.model_file = os.path.join(model_path, model_file)
        print(" > Loading TTS model ...")
        print(" | > model config: ", tts_config)
        print(" | > model file: ", model_file)
        self.tts_config = load_config(tts_config)
        self.use_phonemes = self.tts_config.use_phonemes
        self.ap = AudioProcessor(**self.tts_config.audio)
        c = self.tts_config
        if self.use_phonemes:
            self.input_adapter = lambda sen: _text.phoneme_to_sequence(sen, [c.text_cleaner], c.phoneme_language,
                                                                       c.enable_eos_bos_chars)
        else:
            self.input_adapter = lambda sen: _text.text_to_sequence(sen, [c.text_cleaner])
        self.input_size = _text.num_chars(c)
        self.tts_model = load_model(c, self.model_file)
        self.tts_model.decoder.max_decoder_steps = 3000  # server/synthesizer.py:66

    def split_into_sentences(self, text):
        return split_into_sentences(text)

    def save_wav(self, wav, path):
        self.ap.save_wav(np.array(wav), path)

    def sentences(self, text):
        """The sentences Synthesizer.tts synthesises (server/synthesizer.py:130-136): the split,
        or [text + '.'] when nothing splits, without those shorter than 3 characters."""
        sens = self.split_into_sentences(text)
        if len(sens) == 0:
            sens = [text + "."]
        return [s.strip() for s in sens if len(s) >= 3]

    def tts(self, text):
        sens = self.sentences(text)
        adapter = self.input_adapter or (lambda sen: text_to_seqvec(sen, self.tts_config))
        ids = [np.asarray(adapter(s)) for s in sens]
        wavs = []
        if ids:
            outs, _ = synthesize_batch(self.tts_model, self.ap, ids, seed=self.seed, phase="numpy")
            for w in outs:
                wavs += list(w)
                wavs += [0] * 10000  # server/synthesizer.py:158
        out = io.BytesIO()
        self.save_wav(wavs, out)
        return out
