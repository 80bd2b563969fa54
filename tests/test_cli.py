"""synthesize.py CLI surface (reference synthesize.py:41-146) and the config-built Synthesizer
(server/synthesizer.py:29-66).  CPU: argument parsing, the output file naming and the weights-only
checkpoint load; GPU: the CLI end to end on a generated checkpoint, and Synthesizer(config) vs the
Synthesizer built from parts."""
import os

import numpy as np
import pytest
import torch

from conftest import golden, golden_flags, load_pkg, weights_mod
from oracle.griffin_lim_oracle import AudioOracle
from oracle.tacotron2_oracle import Tacotron2Oracle

CHAR_CFG = {"use_phonemes": False, "text_cleaner": "basic_cleaners"}


def _write_model_files(tmp_path, seed=3):
    """A character-input Tacotron2 config (the shipped configs use phonemes, whose front-end needs
    espeak) and a checkpoint {'model': state_dict} of generator weights, as train.py saves them."""
    import json
    gu = load_pkg("generic_utils")
    txt = load_pkg("text")
    src = os.path.join(gu.CONFIG_DIR, "config_tacotron2.json")
    cfg = gu.load_config(src)
    cfg.update(CHAR_CFG)
    cfg_path = tmp_path / "config.json"
    cfg_path.write_text(json.dumps(cfg))
    n = txt.num_chars(cfg)
    sd = {k: torch.from_numpy(v) for k, v in weights_mod().tacotron2_weights(seed, num_chars=n).items()}
    ckpt = tmp_path / "checkpoint_1.pth.tar"
    torch.save({"model": sd, "step": 1}, ckpt)
    return cfg_path, ckpt, sd


def test_output_file_naming():
    syn = load_pkg("synthesize")
    assert syn.output_file("Hello, world! It's me.", "/out") == "/out/Hello_world_Its_me.wav"
    assert syn.output_file("a_b c-d", "o") == os.path.join("o", "a_b_cd.wav")


def test_parser_matches_reference_options():
    p = load_pkg("synthesize").build_parser()
    a = p.parse_args(["hi there", "c.json", "m.pth", "out"])
    assert (a.text, a.config_path, a.model_path, a.out_path) == ("hi there", "c.json", "m.pth", "out")
    assert a.use_cuda is False and a.vocoder_path == "" and a.batched_vocoder is True
    # argparse type=bool, as in the reference: any non-empty string is True
    assert p.parse_args(["t", "c", "m", "o", "--use_cuda", "False"]).use_cuda is True


def test_checkpoint_is_loaded_weights_only(tmp_path):
    _, ckpt, sd = _write_model_files(tmp_path)
    cp = load_pkg("synthesize").load_checkpoint(str(ckpt))
    assert set(cp["model"]) == set(sd) and torch.equal(cp["model"]["embedding.weight"], sd["embedding.weight"])

    class _Evil:
        def __reduce__(self):
            return (os.system, ("true",))

    bad = tmp_path / "bad.pth"
    torch.save({"model": _Evil()}, bad)
    with pytest.raises(Exception):
        load_pkg("synthesize").load_checkpoint(str(bad))


@pytest.mark.gpu
def test_cli_end_to_end_vs_oracle_chain(tmp_path, audio_cfg):
    """python -m your-voice-tts_amd.synthesize text config model out: the file is named as
    synthesize.py:142-144 names it and holds the oracle chain's int16 samples (same numpy phases,
    forward_attn_mask forced on as :86 does) within 2 LSB."""
    import scipy.io.wavfile
    syn = load_pkg("synthesize")
    txt = load_pkg("text")
    cfg_path, ckpt, sd = _write_model_files(tmp_path)
    out_dir = tmp_path / "out"
    out_dir.mkdir()
    text = "Hello world, it works."
    np.random.seed(123)
    path = syn.main([text, str(cfg_path), str(ckpt), str(out_dir)])
    assert path == str(out_dir / "Hello_world_it_works.wav") and os.path.exists(path)
    sr, pcm = scipy.io.wavfile.read(path)
    assert sr == 22050 and pcm.dtype == np.int16
    fl = golden_flags(golden("t2_fwdmask_L100"))
    assert fl["forward_attn_mask"]
    o = Tacotron2Oracle({k: v.numpy() for k, v in sd.items()}, dtype=np.float32, **fl)
    ids = np.asarray(txt.text_to_sequence(text, ["basic_cleaners"]))
    ref = o.inference(ids)
    np.random.seed(123)
    wav = AudioOracle(**audio_cfg).inv_mel_spectrogram(ref["mel_post"].T)
    ref_pcm = AudioOracle.wav_to_int16(wav)
    assert pcm.shape == ref_pcm.shape
    assert np.abs(pcm.astype(np.int32) - ref_pcm).max() <= 2


@pytest.mark.gpu
def test_synthesizer_from_server_config_matches_parts(tmp_path, audio_cfg):
    """Synthesizer(config) (server/synthesizer.py:30-66: tts_path / tts_file / tts_config, weights
    from the checkpoint, 3000-step cap) gives bitwise the request output of the Synthesizer built
    from the same model parts."""
    import json
    cfg_path, ckpt, sd = _write_model_files(tmp_path)
    synth = load_pkg("synthesis")
    gu = load_pkg("generic_utils")
    audio = load_pkg("audio")
    txt = load_pkg("text")
    conf = tmp_path / "conf.json"
    conf.write_text('{"tts_path": "%s", // model folder\n "tts_file": "%s", "tts_config": "config.json",\n'
                    ' "wavernn_lib_path": "", "use_cuda": true, "port": 5002}' % (tmp_path, ckpt.name))
    s = synth.Synthesizer(gu.load_config(str(conf)))
    assert s.tts_model.decoder.max_decoder_steps == 3000 and s.tts_model.flags["forward_attn_mask"] is False
    text = "The quick brown fox. It jumped!"
    np.random.seed(9)
    a = s.tts(text).getvalue()
    C = gu.load_config(str(cfg_path))
    m = gu.setup_model(txt.num_chars(C), C)
    m.load_state_dict(sd)
    m.cuda()
    s2 = synth.Synthesizer(m, audio.AudioProcessor(**C.audio), C,
                           input_adapter=lambda x: txt.text_to_sequence(x, ["basic_cleaners"]))
    np.random.seed(9)
    b = s2.tts(text).getvalue()
    assert a == b and len(a) > 44
    assert json.loads(cfg_path.read_text())["use_phonemes"] is False
