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
import scipy.io.wavfile
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


def _resident_batch(model, ids_list):
    """Whether the whole request decodes in one call on a resident decoder (the batch-1 one, or the
    batch one for 2..max sentences, tts_decoder_resident_limits)."""
    Lmax = max(len(x) for x in ids_list)
    mb, ml = model.resident_limits(Lmax)
    return len(ids_list) <= mb and Lmax <= ml


def _serial_eligible(model, ids_list):
    """Whether a request decodes serially on the resident batch-1 decoder: 2..SERIAL_RESIDENT_MAX
    sentences the batch decoder does not take, each within the length the handle's resident
    decoder serves now (tts_decoder_resident_limits: no hard-coded limit here)."""
    B = len(ids_list)
    if B < 2 or B > SERIAL_RESIDENT_MAX:
        return False
    Lmax = max(len(x) for x in ids_list)
    mb, ml = model.resident_limits(Lmax)
    return mb == 1 and Lmax <= ml


def _stack(outs, B):
    """Per-call inference_batch dicts (in sentence order) -> the batch dict inference_batch returns
    for the whole request: mel / mel_post [B, T, 80], align [B, S, Lmax], stop [B, S], zero-padded."""
    frames = [f for o in outs for f in o["frames"]]
    steps = [n for o in outs for n in o["steps"]]
    lens = [n for o in outs for n in o["lens"]]
    T, S, Lmax = max(frames), max(steps), max(lens)
    dev = outs[0]["mel_post"].device
    res = dict(mel=torch.zeros(B, T, outs[0]["mel"].shape[2], device=dev),
               mel_post=torch.zeros(B, T, outs[0]["mel_post"].shape[2], device=dev),
               align=torch.zeros(B, S, Lmax, device=dev), stop=torch.zeros(B, S, device=dev))
    b = 0
    for o in outs:
        for k in range(len(o["frames"])):
            t, n, L = o["frames"][k], o["steps"][k], o["lens"][k]
            res["mel"][b, :t] = o["mel"][k, :t]
            res["mel_post"][b, :t] = o["mel_post"][k, :t]
            res["align"][b, :n, :L] = o["align"][k, :n, :L]
            res["stop"][b, :n] = o["stop"][k, :n]
            b += 1
    res.update(frames=frames, steps=steps, lens=lens)
    return res


def _decode(model, ids_list, speaker_ids=None):
    """Tacotron2 decode of a request: serial resident calls below the crossover, else one batch.
    Both dispatches return inference_batch's dict; ``decoder_timings`` lists each call's timing."""
    B = len(ids_list)
    if not _serial_eligible(model, ids_list):
        out = model.inference_batch(ids_list, speaker_ids=speaker_ids)
        out["dispatch"] = {2: "batch-resident", 1: "batch-resident"}.get(model.last_timing.get("resident_kind", 0), "batch")
        out["decoder_timings"] = [dict(model.last_timing)]
        return out
    from .tacotron2 import _speaker_array
    spk = None if speaker_ids is None else _speaker_array(speaker_ids, B)
    outs, timings = [], []
    for b, x in enumerate(ids_list):
        outs.append(model.inference_batch([x], speaker_ids=None if spk is None else spk[b:b + 1]))
        timings.append(dict(model.last_timing))
        if not model.last_timing.get("resident") and b + 1 < B:
            # this call fell off the resident path (placement, a long sentence): the rest as one
            # batch is cheaper than more multi-launch batch-1 calls
            outs.append(model.inference_batch(ids_list[b + 1:], speaker_ids=None if spk is None else spk[b + 1:]))
            timings.append(dict(model.last_timing))
            break
    out = _stack(outs, B)
    out["dispatch"] = "serial-resident"
    out["decoder_timings"] = timings
    # the request's decoder loop time is the sum of its calls'
    model.last_timing = dict(timings[-1], decoder_loop_ms=sum(t.get("decoder_loop_ms", 0.0) for t in timings),
                             decoder_steps_run=sum(t.get("decoder_steps_run", 0) for t in timings),
                             resident=all(t.get("resident") for t in timings))
    return out


@torch.no_grad()
def synthesize_batch(model, ap: AudioProcessor, ids_list, speaker_ids=None, seed=0, phase="device",
                     iters=None, keep_outputs=False, style_mel=None, to_host=True):
    """ids -> encoder -> HIP decoder -> HIP postnet -> HIP Griffin-Lim for a ragged batch.

    phase: "device" draws the initial GL phases on the GPU from ``seed``; "numpy" gives every
    sentence numpy's np.random.rand(1025, T_b) draw in batch order, as the reference does when it
    synthesises the sentences one after another (utils/audio.py:183) -- continued on the device from
    numpy's global state (ap.numpy_phases, phase_mt.hip), which is left where those draws would
    leave it.  Returns (wavs: list of float64 numpy arrays, or None with to_host=False, info dict;
    info["wav_dev"] is the CUDA fp64 [B, N] waveform batch with keep_outputs or to_host=False)."""
    linear = hasattr(model, "linear_dim")  # Tacotron / TacotronGST: linear-spectrogram GL
    if linear:
        out = model.inference_batch(ids_list, speaker_ids=speaker_ids, style_mel=style_mel)
    else:  # (keep_outputs or not: the same dispatch, so a sharded rank decodes as the single process does)
        out = _decode(model, ids_list, speaker_ids)
    frames = out["frames"]
    mel_post = out["linear"] if linear else out["mel_post"]
    mode = _native.TTS_GL_FROM_LINEAR if linear else _native.TTS_GL_FROM_MEL
    if phase == "numpy":
        with ap.numpy_phases():
            wav = ap.griffin_lim_batch(mel_post, frames, mode=mode, iters=iters)
    elif phase == "device":
        wav = ap.griffin_lim_batch(mel_post, frames, mode=mode, seed=seed, iters=iters)
    else:
        raise ValueError(f"phase must be 'device' or 'numpy', not {phase!r}")
    lens = [ap.hop_length * (T - 1) for T in frames]
    info = dict(frames=frames, steps=out["steps"], samples=lens, decoder_dispatch=out.get("dispatch", "batch"),
                **model.last_timing, **ap.last_gl_timing())
    if keep_outputs:
        info.update(out)
    if keep_outputs or not to_host:
        info["wav_dev"] = wav
    if not to_host:
        return None, info
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

    def synthesize(self, ids):
        """The waveforms of a request's sentences, on the device: (CUDA fp64 [B, pitch], samples per
        sentence).  Initial phases from numpy's global stream (the caller is inside
        ap.numpy_phases()).  Tacotron2 requests of up to SERIAL_RESIDENT_MAX sentences run one
        tts_synth_run per sentence (encoder -> resident decoder -> postnet -> Griffin-Lim in one
        native call each); larger ones, and the Tacotron family, as one batch (synthesize_batch)."""
        model, ap = self.tts_model, self.ap
        if not hasattr(model, "linear_dim") and len(ids) > 1 and _resident_batch(model, ids):
            # the resident batch decoder: the whole request in one tts_synth_run
            buf = torch.empty(model.native_wav_capacity(ap, len(ids)), dtype=torch.float64, device="cuda")
            wav, frames = model.synthesize_native(ids, ap, sync=True, out=buf)
            return wav, [ap.hop_length * (T - 1) for T in frames]
        if not hasattr(model, "linear_dim") and (len(ids) == 1 or _serial_eligible(model, ids)):
            cap = model.native_wav_capacity(ap, 1)
            buf = torch.empty(len(ids), cap, dtype=torch.float64, device="cuda")
            lens = []
            for b, x in enumerate(ids):
                # sync: the next sentence's resident launch must not share the device with this one's
                # Griffin-Lim (and the numpy stream stays in sentence order)
                _, frames = model.synthesize_native([x], ap, sync=True, out=buf[b])
                lens.append(ap.hop_length * (frames[0] - 1))
            return buf, lens
        _, info = synthesize_batch(model, ap, ids, seed=self.seed, phase="numpy", to_host=False)
        return info["wav_dev"], info["samples"]

    def tts(self, text):
        """server/synthesizer.py:128-162: split, synthesise every sentence, join them with 10 000
        zeros after each, peak-normalise to int16 and return the wav in a BytesIO.  The waveforms stay
        on the device until the int16 join (tts_gl_save_pcm16: the reference's Python-list join and
        save_wav conversion, bytes equal); the phases are numpy's global stream continued on the
        device (the reference's per-sentence np.random.rand draws, utils/audio.py:183)."""
        sens = self.sentences(text)
        adapter = self.input_adapter or (lambda sen: text_to_seqvec(sen, self.tts_config))
        ids = [np.asarray(adapter(s)) for s in sens]
        out = io.BytesIO()
        if not ids:  # the reference's save_wav([]) raises on the empty maximum, so does this
            self.save_wav([], out)
            return out
        with self.ap.numpy_phases():
            wav, lens = self.synthesize(ids)
        pcm = self.ap.pcm16_join(wav, lens, gap=10000)  # server/synthesizer.py:158
        scipy.io.wavfile.write(out, self.ap.sample_rate, pcm)
        return out
