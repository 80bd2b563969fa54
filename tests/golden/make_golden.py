"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Run in the build container only (needs /root/reference; nothing here runs on the GPU box):

    python tests/golden/make_golden.py

Model half (t2_*.npz): the reference ``Tacotron2`` (``models/tacotron2.py``) is imported from
/root/reference with its text front-end dependencies (phonemizer, unidecode — absent from the
image and not on the numeric path) stubbed in ``sys.modules``; it is built with
``utils.generic_utils.setup_model`` from ``config_tacotron2.json`` plus per-case flag
overrides, loaded with weights from ``weights.py``'s deterministic generator, put in eval
mode and run through ``inference`` on seeded ids.  Inputs and outputs are saved.

Tacotron / TacotronGST half (gst_*.npz, taco_*.npz): the reference ``Tacotron`` /
``TacotronGST`` (``models/tacotron.py``, ``models/tacotrongst.py``) built the same way from
``config_tacotron.json`` / ``config_tacotron_gst.json`` (+ per-case overrides), with
``weights.tacotron_gst_weights`` and, for GST cases, a seeded synthetic style mel.

GL half (gl_*.npz): the reference ``AudioProcessor`` (``utils/audio.py``) is imported with
``librosa``/``soundfile`` replaced by the oracle's librosa-0.6.2 restatement (librosa is
absent), and ``np.complex`` aliased to ``complex`` (removed in numpy>=1.24; same meaning).  This
pins the reference's own glue (denormalise, dB->amp, pinv, power, GL loop order, lfilter)
but NOT librosa's internals, which stay unpinned.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


weights = _load("yvtts_weights", os.path.join(REPO, "your-voice-tts_amd", "weights.py"))
sys.path.insert(0, REPO)
from oracle import griffin_lim_oracle as glo  # noqa: E402


def _stub_text_deps():
    for m in ("phonemizer", "phonemizer.phonemize", "unidecode"):
        sys.modules.setdefault(m, types.ModuleType(m))
    sys.modules["phonemizer"].phonemize = lambda *a, **k: ""
    sys.modules["phonemizer.phonemize"].phonemize = lambda *a, **k: ""
    sys.modules["unidecode"].unidecode = lambda s: s


def _stub_audio_deps():
    lib = types.ModuleType("librosa")
    lib.filters = types.SimpleNamespace(
        mel=lambda sr, n_fft, n_mels=128, fmin=0.0, fmax=None: glo.mel_filters(sr, n_fft, n_mels, fmin, fmax))
    lib.stft = lambda y, n_fft, hop_length, win_length: glo.stft(y, n_fft, hop_length, win_length)
    lib.istft = lambda y, hop_length, win_length: glo.istft(y, hop_length, win_length)
    sys.modules["librosa"] = lib
    sys.modules["soundfile"] = types.ModuleType("soundfile")
    if not hasattr(np, "complex"):
        np.complex = complex


CASES = [
    # name, L, id seed, overrides of config_tacotron2.json (+ forward_attn_mask from synthesize.py:86)
    ("t2_fwdmask_L12", 12, 11, dict(forward_attn_mask=True), None),
    ("t2_fwdmask_L40", 40, 12, dict(forward_attn_mask=True), None),
    ("t2_fwdmask_L100", 100, 1, dict(forward_attn_mask=True), None),
    ("t2_nomask_L12", 12, 13, dict(forward_attn_mask=False), 60),
    ("t2_loc_softmax_L20", 20, 14,
     dict(location_attn=True, attention_norm="softmax", use_forward_attn=False, forward_attn_mask=False), 50),
    ("t2_loc_fwd_ta_L24", 24, 15,
     dict(location_attn=True, use_forward_attn=True, transition_agent=True, forward_attn_mask=True), 90),
    ("t2_win_fwdmask_L16", 16, 16, dict(windowing=True, forward_attn_mask=True), 60),
    ("t2_win_softmax_L16", 16, 17,
     dict(windowing=True, attention_norm="softmax", use_forward_attn=False, forward_attn_mask=False), 40),
]


LONG_CASES = [
    # round 5: the resident decoder's general attention form at full length.  Synthesizer.tts()'s
    # configuration is config_tacotron2.json as it is (forward attention, sigmoid, mask OFF,
    # server/synthesizer.py:55); the constructor default is location-sensitive + softmax
    # (models/tacotron2.py:17,23); both run to their step cap under random weights.
    ("t2_nomask_L100", 100, 1, dict(), None),
    ("t2_loc_softmax_L100", 100, 2,
     dict(location_attn=True, attention_norm="softmax", use_forward_attn=False, forward_attn_mask=False), 300),
    ("t2_loc_fwd_ta_L100", 100, 3,
     dict(location_attn=True, use_forward_attn=True, transition_agent=True, forward_attn_mask=False), 300),
]


# round 6: Synthesizer.tts()'s configuration at its real step cap (server/synthesizer.py:66 sets
# max_decoder_steps = 3000; layers/tacotron2.py:259-277 stops there): past the resident decoder's
# 2048-step tag wrap, pinned to the reference itself (VERDICT r5 missing 3)
CAP3000_CASES = [("t2_nomask_L100_cap3000", 100, 1, dict(), 3000)]


def make_model_fixtures(cases=CASES):
    import torch
    _stub_text_deps()
    sys.path.insert(0, REF)
    from utils.generic_utils import load_config, setup_model
    torch.set_num_threads(os.cpu_count())
    for name, L, seed, over, cap in cases:
        C = load_config(os.path.join(REF, "config_tacotron2.json"))
        C.num_speakers = 0
        C.update(over)
        model = setup_model(130, 0, C)
        sd = weights.tacotron2_weights(0, num_chars=130, location_attn=C.location_attn,
                                       trans_agent=C.transition_agent)
        ref_sd = model.state_dict()
        assert list(ref_sd.keys()) == list(sd.keys()), (set(ref_sd) ^ set(sd))
        model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        model.eval()
        if cap is not None:
            model.decoder.max_decoder_steps = cap
        ids = weights.synthetic_ids(L, seed)
        with torch.no_grad():
            x = torch.from_numpy(ids).unsqueeze(0)
            enc = model.encoder.inference(model.embedding(x).transpose(1, 2))
            mel, mel_post, align, stop = model.inference(x)
        flags = dict(attn_norm=C.attention_norm, forward_attn=C.use_forward_attn,
                     trans_agent=C.transition_agent, forward_attn_mask=C.forward_attn_mask,
                     location_attn=C.location_attn, attn_win=C.windowing,
                     max_decoder_steps=model.decoder.max_decoder_steps)
        np.savez_compressed(
            os.path.join(HERE, name + ".npz"), ids=ids, enc=enc[0].numpy(), mel=mel[0].numpy(),
            mel_post=mel_post[0].numpy(), align=align[0].numpy(), stop=stop[0, :, 0].numpy(),
            flags=np.array(repr(flags)))
        print(f"{name}: L={L} T={mel.shape[1]} flags={flags}")


SPEAKER_CASES = [
    # name, L, id seed, speaker id (of 4): Tacotron2 with speaker embeddings (models/tacotron2.py:32-34,
    # 91-100) under the synthesis attention configuration (forward attention + mask)
    ("t2spk_fwdmask_L24_s2", 24, 21, 2),
    ("t2spk_fwdmask_L40_s0", 40, 22, 0),
]


def make_speaker_fixtures():
    import torch
    _stub_text_deps()
    sys.path.insert(0, REF)
    from utils.generic_utils import load_config, setup_model
    torch.set_num_threads(os.cpu_count())
    for name, L, seed, spk in SPEAKER_CASES:
        C = load_config(os.path.join(REF, "config_tacotron2.json"))
        C.num_speakers = 4
        C.forward_attn_mask = True
        model = setup_model(130, 4, C)
        sd = weights.tacotron2_weights(0, num_chars=130, num_speakers=4)
        ref_sd = model.state_dict()
        assert list(ref_sd.keys()) == list(sd.keys()), (set(ref_sd) ^ set(sd))
        model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        model.eval()
        ids = weights.synthetic_ids(L, seed)
        with torch.no_grad():
            x = torch.from_numpy(ids).unsqueeze(0)
            sid = torch.tensor([spk])
            enc = model._add_speaker_embedding(model.encoder.inference(model.embedding(x).transpose(1, 2)), sid)
            mel, mel_post, align, stop = model.inference(x, speaker_ids=sid)
        flags = dict(attn_norm=C.attention_norm, forward_attn=C.use_forward_attn,
                     trans_agent=C.transition_agent, forward_attn_mask=C.forward_attn_mask,
                     location_attn=C.location_attn, attn_win=C.windowing,
                     max_decoder_steps=model.decoder.max_decoder_steps)
        np.savez_compressed(
            os.path.join(HERE, name + ".npz"), ids=ids, speaker_id=np.array(spk), enc=enc[0].numpy(),
            mel=mel[0].numpy(), mel_post=mel_post[0].numpy(), align=align[0].numpy(), stop=stop[0, :, 0].numpy(),
            flags=np.array(repr(flags)))
        print(f"{name}: L={L} speaker={spk} T={mel.shape[1]}")


def make_prenet_bn_fixtures():
    """Tacotron2 with prenet_type "bn" (common_layers.py:27-52, 55-83; eval-mode BatchNorm1d)."""
    import torch
    _stub_text_deps()
    sys.path.insert(0, REF)
    from utils.generic_utils import load_config, setup_model
    torch.set_num_threads(os.cpu_count())
    for name, L, seed in (("t2bn_fwdmask_L24", 24, 31), ("t2bn_fwdmask_L40", 40, 32)):
        C = load_config(os.path.join(REF, "config_tacotron2.json"))
        C.num_speakers = 0
        C.forward_attn_mask = True
        C.prenet_type = "bn"
        model = setup_model(130, 0, C)
        sd = weights.tacotron2_weights(0, num_chars=130, prenet_bn=True)
        ref_sd = model.state_dict()
        assert list(ref_sd.keys()) == list(sd.keys()), (set(ref_sd) ^ set(sd))
        model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        model.eval()
        ids = weights.synthetic_ids(L, seed)
        with torch.no_grad():
            x = torch.from_numpy(ids).unsqueeze(0)
            enc = model.encoder.inference(model.embedding(x).transpose(1, 2))
            mel, mel_post, align, stop = model.inference(x)
        flags = dict(attn_norm=C.attention_norm, forward_attn=C.use_forward_attn,
                     trans_agent=C.transition_agent, forward_attn_mask=C.forward_attn_mask,
                     location_attn=C.location_attn, attn_win=C.windowing,
                     max_decoder_steps=model.decoder.max_decoder_steps)
        np.savez_compressed(
            os.path.join(HERE, name + ".npz"), ids=ids, enc=enc[0].numpy(), mel=mel[0].numpy(),
            mel_post=mel_post[0].numpy(), align=align[0].numpy(), stop=stop[0, :, 0].numpy(),
            flags=np.array(repr(flags)))
        print(f"{name}: L={L} T={mel.shape[1]}")


# name, config file, L, id seed, num_speakers, speaker id, (style frames, style seed) or None,
# max_decoder_steps, overrides.  Small L exercise the stop rule (layers/tacotron.py:464-469): L=2
# stops on the stop token at t=1, L=4/10 on the alignment tail, L=24 runs into the cap.
TACO_CASES = [
    ("gst_L24_style_spk", "config_tacotron_gst.json", 24, 21, 4, 1, (60, 31), 20, {}),
    ("gst_L10_nostyle", "config_tacotron_gst.json", 10, 50, 0, None, None, 40, {}),
    ("gst_L4_style", "config_tacotron_gst.json", 4, 44, 0, None, (33, 32), 40, {}),
    ("gst_L2_nostyle", "config_tacotron_gst.json", 2, 42, 0, None, None, 40, {}),
    ("taco_L10_loc_ta", "config_tacotron.json", 10, 50, 0, None, None, 40, dict(location_attn=True)),
    ("taco_L12_softmax", "config_tacotron.json", 12, 23, 0, None, None, 16,
     dict(attention_norm="softmax", use_forward_attn=False, transition_agent=False)),
]
# prenet_type "bn" (common_layers.py:28-52, 66-70) on the Tacotron decoder prenet ("taco_bn" target)
TACO_BN_CASES = [
    ("gst_L10_prenetbn", "config_tacotron_gst.json", 10, 51, 0, None, (40, 33), 30, dict(prenet_type="bn")),
    ("taco_L12_prenetbn", "config_tacotron.json", 12, 52, 0, None, None, 30, dict(prenet_type="bn")),
]


def make_taco_fixtures(cases=TACO_CASES):
    import torch
    _stub_text_deps()
    sys.path.insert(0, REF)
    from utils.generic_utils import load_config, setup_model
    torch.set_num_threads(os.cpu_count())
    for name, cfgname, L, seed, nspk, spk, style, cap, over in cases:
        C = load_config(os.path.join(REF, cfgname))
        C.update(over)
        gst = C.model == "TacotronGST"
        model = setup_model(130, nspk, C)
        sd = weights.tacotron_gst_weights(0, num_chars=130, num_speakers=nspk, r=C.r, memory_size=C.memory_size,
                                          location_attn=C.location_attn, trans_agent=C.transition_agent, gst=gst,
                                          prenet_bn=C.prenet_type == "bn")
        assert list(model.state_dict().keys()) == list(sd.keys()), (set(model.state_dict()) ^ set(sd))
        model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        model.eval()
        model.decoder.max_decoder_steps = cap
        ids = weights.synthetic_ids(L, seed)
        x = torch.from_numpy(ids)[None]
        sm = weights.synthetic_style_mel(*style)[None] if style else None
        sid = torch.tensor([spk]) if spk is not None else None
        with torch.no_grad():
            enc = model._add_speaker_embedding(model.encoder(model.embedding(x)), sid)
            extra = {}
            if sm is not None:
                g = model.gst(torch.from_numpy(sm))
                enc = enc + g.expand(-1, L, -1)
                extra = dict(style_mel=sm[0], gst=g[0, 0].numpy())
            if gst:
                mel, lin, align, stop = model.inference(x, speaker_ids=sid, style_mel=(
                    torch.from_numpy(sm) if sm is not None else None))
            else:
                mel, lin, align, stop = model.inference(x, speaker_ids=sid)
        flags = dict(model=C.model, r=C.r, memory_size=C.memory_size, attn_norm=C.attention_norm,
                     forward_attn=C.use_forward_attn, trans_agent=C.transition_agent,
                     forward_attn_mask=C.forward_attn_mask, location_attn=C.location_attn, attn_win=C.windowing,
                     max_decoder_steps=cap, num_speakers=nspk)
        if C.prenet_type != "original":
            flags["prenet_type"] = C.prenet_type
        np.savez_compressed(
            os.path.join(HERE, name + ".npz"), ids=ids, enc=enc[0].numpy(), mel=mel[0].numpy(),
            linear=lin[0].numpy(), align=align[0].numpy(), stop=stop[0].numpy(),
            speaker_id=np.array(-1 if spk is None else spk), flags=np.array(repr(flags)), **extra)
        print(f"{name}: L={L} steps={align.shape[1]} frames={mel.shape[1]} flags={flags}")


def make_truncated_fixture():
    """Tacotron2.inference_truncated over three consecutive texts (continuous mode,
    models/tacotron2.py:75-89): encoder BiLSTM state and decoder states carry over."""
    import torch
    _stub_text_deps()
    sys.path.insert(0, REF)
    from utils.generic_utils import load_config, setup_model
    C = load_config(os.path.join(REF, "config_tacotron2.json"))
    C.num_speakers = 0
    C.forward_attn_mask = True
    model = setup_model(130, 0, C)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in weights.tacotron2_weights(0, num_chars=130).items()})
    model.eval()
    out = {}
    for i, (L, seed) in enumerate(((12, 61), (9, 62), (15, 63))):
        ids = weights.synthetic_ids(L, seed)
        with torch.no_grad():
            mel, mel_post, align, stop = model.inference_truncated(torch.from_numpy(ids)[None])
        out.update({f"ids{i}": ids, f"mel{i}": mel[0].numpy(), f"mel_post{i}": mel_post[0].numpy(),
                    f"align{i}": align[0].numpy(), f"stop{i}": stop[0, :, 0].numpy()})
        print(f"trunc_t2_3texts text {i}: L={L} T={mel.shape[1]}")
    flags = dict(attn_norm=C.attention_norm, forward_attn=C.use_forward_attn, trans_agent=C.transition_agent,
                 forward_attn_mask=C.forward_attn_mask, location_attn=C.location_attn, attn_win=C.windowing,
                 max_decoder_steps=model.decoder.max_decoder_steps)
    np.savez_compressed(os.path.join(HERE, "trunc_t2_3texts.npz"), flags=np.array(repr(flags)), **out)


TF_CASES = [
    # name, L, id seed, teacher frames, teacher seed, config overrides (+ forward_attn_mask)
    ("tf_fwdmask_L12", 12, 11, 40, 71, dict(forward_attn_mask=True)),
    ("tf_loc_softmax_L20", 20, 14, 30, 72,
     dict(location_attn=True, attention_norm="softmax", use_forward_attn=False, forward_attn_mask=False)),
    ("tf_win_fwdmask_L16", 16, 16, 24, 73, dict(windowing=True, forward_attn_mask=True)),
]


def make_teacher_fixtures():
    """Teacher-forced Decoder.forward(inputs, memories, mask=None) (layers/tacotron2.py:227-247) of the
    reference in eval mode on seeded U[0,1) teacher mels, plus Postnet + residual on its output
    (models/tacotron2.py:56-57).  (The reference's Tacotron2.forward itself cannot run on torch >= 1.2:
    common_layers.py:234 computes `1 - mask` on a bool mask; with mask=None the decoder runs.)"""
    import torch
    _stub_text_deps()
    sys.path.insert(0, REF)
    from utils.generic_utils import load_config, setup_model
    for name, L, seed, T, tseed, over in TF_CASES:
        C = load_config(os.path.join(REF, "config_tacotron2.json"))
        C.num_speakers = 0
        C.update(over)
        model = setup_model(130, 0, C)
        sd = weights.tacotron2_weights(0, num_chars=130, location_attn=C.location_attn, trans_agent=C.transition_agent)
        model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        model.eval()
        ids = weights.synthetic_ids(L, seed)
        teacher = np.random.Generator(np.random.PCG64(tseed)).uniform(0, 1, size=(T, 80)).astype(np.float32)
        with torch.no_grad():
            x = torch.from_numpy(ids).unsqueeze(0)
            enc = model.encoder.inference(model.embedding(x).transpose(1, 2))
            mel, stop, align = model.decoder(enc, torch.from_numpy(teacher)[None], None)
            mel_post = mel + model.postnet(mel)
        flags = dict(attn_norm=C.attention_norm, forward_attn=C.use_forward_attn, trans_agent=C.transition_agent,
                     forward_attn_mask=C.forward_attn_mask, location_attn=C.location_attn, attn_win=C.windowing,
                     max_decoder_steps=model.decoder.max_decoder_steps)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), ids=ids, enc=enc[0].numpy(), teacher=teacher,
                            mel=mel[0].numpy(), mel_post=mel_post[0].numpy(), stop=stop[0].numpy(),
                            align=align[0].numpy(), flags=np.array(repr(flags)))
        print(f"{name}: L={L} T={T} mel {tuple(mel.shape)} stop {tuple(stop.shape)} align {tuple(align.shape)}")


TEXTS = ["Hello world.", "It took me quite a long time to develop a voice, and now that I have it I'm not going "
         "to be silent.", "  Mixed   CASE\twhitespace;  (and) punctuation: ok?  ", "Turn left on {HH AW1 S S T AH0 N} Street.",
         "Numbers 1234 & symbols #%* are dropped!"]


def make_text_fixture():
    """text_to_sequence / sequence_to_text with basic_cleaners (utils/text/__init__.py:77-112) and
    the symbol tables (utils/text/symbols.py), from the reference module itself."""
    _stub_text_deps()
    sys.path.insert(0, REF)
    import importlib
    text = importlib.import_module("utils.text")
    symbols = importlib.import_module("utils.text.symbols")
    seqs = [np.array(text.text_to_sequence(t, ["basic_cleaners"]), dtype=np.int64) for t in TEXTS]
    back = [text.sequence_to_text(list(s)) for s in seqs]
    np.savez_compressed(os.path.join(HERE, "text_basic.npz"), texts=np.array(TEXTS), back=np.array(back),
                        symbols=np.array(symbols.symbols), phonemes=np.array(symbols.phonemes),
                        **{f"seq{i}": s for i, s in enumerate(seqs)})
    print("text_basic:", [len(s) for s in seqs])


SPLIT_TEXTS = [
    "Hello world. This is a test.",
    "Mr. Smith went to Washington. He arrived at 5 p.m. and left!",
    "Dr. Jones has a Ph.D. in physics. She works at Acme Inc. They build rockets.",
    "The U.S.A. is large. The U.K. is not. But the E.U. is.",
    "Visit www.example.com or mail.org today. It's free?",
    "He said \"stop.\" Then he left. \"Why?\" she asked! \"Go!\" he replied.",
    "Curly quotes: “Fine.” Next one. Jr. was here. Mrs. Brown Jr. said hi.",
    "No terminal punctuation here",
    "Multi\nline\ntext. Second line! Third?",
    "A. B. C. single letters. J.R.R. Tolkien wrote books. It was good.",
    "Acme Co. However we knew. Ltd. is short. St. Louis is a city.",
    "Ellipsis... and more... done.",
    "ok. no. x. abc.",
    "",
    "   ",
    "It took me quite a long time to develop a voice, and now that I have it I'm not going to be silent.",
]


def make_split_fixture():
    """Synthesizer.split_into_sentences (server/synthesizer.py:102-126) run by the reference module
    itself on a corpus of abbreviations, acronyms, quotes, Ph.D, websites and edge cases; also the
    list Synthesizer.tts keeps (:130-136: [text + '.'] when nothing splits, drop len < 3)."""
    _stub_text_deps()
    _stub_audio_deps()
    sys.path.insert(0, REF)
    srv = _load("ref_server_synthesizer", os.path.join(REF, "server", "synthesizer.py"))
    split = srv.Synthesizer.split_into_sentences
    out = {"texts": np.array(SPLIT_TEXTS, dtype=object).astype(str)}
    for i, t in enumerate(SPLIT_TEXTS):
        sens = split(None, t)
        kept = sens if len(sens) else [t + "."]
        kept = [s.strip() for s in kept if len(s) >= 3]
        out[f"split{i}"] = np.array(sens, dtype=str)
        out[f"kept{i}"] = np.array(kept, dtype=str)
        print(f"split {i}: {sens}")
    np.savez_compressed(os.path.join(HERE, "split_sentences.npz"), **out)


def make_gl_fixtures():
    _stub_text_deps()
    _stub_audio_deps()
    sys.path.insert(0, REF)
    from utils.generic_utils import load_config
    from utils.audio import AudioProcessor
    C = load_config(os.path.join(REF, "config_tacotron2.json"))
    t2 = np.load(os.path.join(HERE, "t2_fwdmask_L12.npz"))
    rng = np.random.Generator(np.random.PCG64(5))
    inputs = {
        "gl_model_mel": t2["mel_post"].T.astype(np.float32),          # [80, T] from the model
        "gl_uniform_mel": rng.uniform(0, 1, size=(80, 30)).astype(np.float32),
    }
    for name, mel in inputs.items():
        for iters in (0, 3, 30):
            audio = dict(C.audio)
            audio["griffin_lim_iters"] = iters
            ap = AudioProcessor(**audio)
            np.random.seed(1234)
            phase_u = np.random.rand(1025, mel.shape[1])
            np.random.seed(1234)
            wav = ap.inv_mel_spectrogram(mel)
            S = ap._mel_to_linear(ap._db_to_amp(ap._denormalize(mel) + ap.ref_level_db)) ** ap.power
            # phase_u is np.random.seed(1234); np.random.rand(1025, T) (legacy MT19937 stream,
            # stable across numpy versions) and is not stored; S only once per input.
            extra = dict(S=S.astype(np.float32)) if iters == 0 else {}
            np.savez_compressed(os.path.join(HERE, f"{name}_it{iters}.npz"), mel=mel,
                                phase_seed=1234, wav=wav, iters=iters, **extra)
            print(f"{name}_it{iters}: T={mel.shape[1]} wav={wav.shape} {wav.dtype}")
    # linear-spectrogram path (Tacotron / TacotronGST, utils/audio.py:154-162)
    lin = rng.uniform(0, 1, size=(1025, 20)).astype(np.float32)
    audio = dict(C.audio)
    audio["griffin_lim_iters"] = 3
    ap = AudioProcessor(**audio)
    np.random.seed(99)
    phase_u = np.random.rand(1025, lin.shape[1])
    np.random.seed(99)
    wav = ap.inv_spectrogram(lin)
    np.savez_compressed(os.path.join(HERE, "gl_linear_it3.npz"), spec=lin, phase_seed=99, wav=wav, iters=3)
    # inverse pre-emphasis (scipy.signal.lfilter is available: this one is fully pinned)
    x = rng.standard_normal(5000).astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "preemph.npz"), x=x, y=ap.apply_inv_preemphasis(x))
    # save_wav int16 conversion (utils/audio.py:56-58), via the reference's own code path
    import scipy.io.wavfile
    import io as _io
    buf = _io.BytesIO()
    ap.save_wav(wav, buf)
    buf.seek(0)
    _, pcm = scipy.io.wavfile.read(buf)
    np.savez_compressed(os.path.join(HERE, "save_wav.npz"), wav=wav, pcm=pcm)
    # forward analysis of compute_style_mel (utils/synthesis.py:28-35): AudioProcessor.melspectrogram
    # on a seeded float64 waveform (1.3 s: chirp + noise), librosa stft/mel via the restatement
    rng2 = np.random.Generator(np.random.PCG64(8))
    n = 28717
    tt = np.arange(n) / 22050.0
    y = 0.3 * np.sin(2 * np.pi * (220 + 800 * tt) * tt) + 0.05 * rng2.standard_normal(n)
    np.savez_compressed(os.path.join(HERE, "melspec.npz"), wav=y, mel=ap.melspectrogram(y))


# tests/test_audio.py:31-55 of the reference: example_1.wav -> melspectrogram -> inv_mel_spectrogram at
# ten (max_norm, signal_norm, symmetric_norm, clip_norm) settings of tests/test_config.json's audio
AUDIO_TEST_SETTINGS = [(1., False, False, False), (1., True, False, False), (1., True, True, False),
                       (1., True, False, True), (1., True, True, True), (4., False, False, False),
                       (4., True, False, False), (4., True, True, False), (4., True, False, True),
                       (4., True, True, True)]


def make_audio_test_fixture():
    """The reference's only natural-speech input (tests/inputs/example_1.wav, a data file its own tests
    hold) through the reference AudioProcessor (utils/audio.py) exactly as tests/test_audio.py:23-55
    drives it, with librosa replaced by the oracle's 0.6.2 restatement (librosa is absent: its
    internals stay unpinned, the reference's glue is pinned) and the GL phases seeded per setting
    (np.random.seed(1000 + i) before inv_mel_spectrogram; the test itself leaves them unseeded).
    load_wav is soundfile's read (float64 = int16 / 32768); soundfile is absent, so the PCM is read
    with scipy.io.wavfile and converted the same way."""
    import json as _json
    import re as _re
    import scipy.io.wavfile
    _stub_text_deps()
    _stub_audio_deps()
    sys.path.insert(0, REF)
    from utils.audio import AudioProcessor
    txt = open(os.path.join(REF, "tests", "test_config.json")).read()
    conf = _json.loads(_re.sub(r"//[^\n]*", "", txt))  # the reference's load_config strips // comments
    sr, pcm = scipy.io.wavfile.read(os.path.join(REF, "tests", "inputs", "example_1.wav"))
    assert pcm.dtype == np.int16 and sr == conf["audio"]["sample_rate"]
    x = pcm.astype(np.float64) / 32768.0
    out = dict(pcm=pcm, audio=np.array(repr(conf["audio"])), settings=np.array(AUDIO_TEST_SETTINGS))
    ap = AudioProcessor(**conf["audio"])
    for i, (max_norm, signal_norm, symmetric_norm, clip_norm) in enumerate(AUDIO_TEST_SETTINGS):
        ap.max_norm, ap.signal_norm, ap.symmetric_norm, ap.clip_norm = max_norm, signal_norm, symmetric_norm, clip_norm
        mel = ap.melspectrogram(x)
        np.random.seed(1000 + i)
        wav_ = ap.inv_mel_spectrogram(mel)
        out[f"mel{i}"] = mel
        out[f"wav{i}"] = wav_.astype(np.float32)  # (rounding 6e-8 relative: far below the 1e-4 check)
        print(f"example_1 setting {i} {AUDIO_TEST_SETTINGS[i]}: mel {mel.shape} [{mel.min():.2f}, {mel.max():.2f}] "
              f"wav {wav_.shape} {wav_.dtype}")
    np.savez_compressed(os.path.join(HERE, "audio_example1.npz"), **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["model", "speakers", "prenet_bn", "taco", "taco_bn", "truncated", "teacher", "text", "split", "gl"]
    if "taco_bn" in which:
        make_taco_fixtures(TACO_BN_CASES)
    if "prenet_bn" in which:
        make_prenet_bn_fixtures()
    if "speakers" in which:
        make_speaker_fixtures()
    if "teacher" in which:
        make_teacher_fixtures()
    if "split" in which:
        make_split_fixture()
    if "model" in which:
        make_model_fixtures()
    if "long" in which:
        make_model_fixtures(LONG_CASES)
    if "cap3000" in which:
        make_model_fixtures(CAP3000_CASES)
    if "audio_test" in which:
        make_audio_test_fixture()
    if "taco" in which:
        make_taco_fixtures()
    if "truncated" in which:
        make_truncated_fixture()
    if "text" in which:
        make_text_fixture()
    if "gl" in which:
        make_gl_fixtures()
