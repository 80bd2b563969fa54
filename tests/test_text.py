"""CPU: the text front-end (utils/text) against the reference's own outputs
(tests/golden/text_basic.npz, made by tests/golden/make_golden.py from the reference module)."""
import numpy as np
import pytest

from conftest import golden, load_pkg

text = load_pkg("text")


def test_symbol_tables_match_reference():
    z = golden("text_basic")
    assert list(z["symbols"]) == text.SYMBOLS
    assert list(z["phonemes"]) == text.PHONEMES


def test_text_to_sequence_basic_cleaners():
    z = golden("text_basic")
    for i, t in enumerate(z["texts"]):
        seq = text.text_to_sequence(str(t), ["basic_cleaners"])
        np.testing.assert_array_equal(seq, z[f"seq{i}"])
        assert text.sequence_to_text(seq) == str(z["back"][i])


def test_missing_frontend_dependencies_raise():
    with pytest.raises(NotImplementedError, match="unidecode"):
        text.text_to_sequence("abc", ["english_cleaners"])
    with pytest.raises(NotImplementedError, match="phonemizer"):
        text.phoneme_to_sequence("abc", ["phoneme_cleaners"], "en-us")
    with pytest.raises(Exception, match="Unknown cleaner"):
        text.text_to_sequence("abc", ["nope"])


def test_split_into_sentences_matches_reference():
    """Synthesizer.split_into_sentences and the sentence list Synthesizer.tts keeps
    (server/synthesizer.py:102-136) vs the reference module run on a hard corpus
    (tests/golden/split_sentences.npz, made by make_golden.py split)."""
    import types
    synth = load_pkg("synthesis")
    z = golden("split_sentences")
    dummy = types.SimpleNamespace(eval=lambda: None, decoder=types.SimpleNamespace(max_decoder_steps=1000))
    s = synth.Synthesizer(dummy, None, None)
    assert dummy.decoder.max_decoder_steps == 3000  # server/synthesizer.py:66
    for i, t in enumerate(z["texts"]):
        t = str(t)
        assert synth.split_into_sentences(t) == [str(x) for x in z[f"split{i}"]], t
        assert s.sentences(t) == [str(x) for x in z[f"kept{i}"]], t
