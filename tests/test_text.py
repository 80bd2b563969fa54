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
