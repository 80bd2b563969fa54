"""Text front-end of the synthesis path (utils/text/__init__.py:77-130, utils/text/cleaners.py,
utils/text/symbols.py): symbol table, ``basic_cleaners``, ``text_to_sequence`` (with ``{ARPAbet}``
spans) and ``sequence_to_text``.  CPU string work, off the GPU path.

``phoneme_to_sequence`` needs phonemizer + espeak and the english/transliteration cleaners need
unidecode / inflect; none of them is installed here, so those raise with the missing dependency
named (callers then pass ids, or an ``input_adapter`` built on the reference's own front-end).
"""
from __future__ import annotations

import re

# symbol inventory (utils/text/symbols.py): pad, eos, bos, the characters, '@' + each phoneme
PAD, EOS, BOS = "_", "~", "^"
CHARACTERS = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz!'(),-.:;? "
PUNCTUATIONS = "!'(),-.:;? "
_IPA_GROUPS = (
    "iyɨʉɯuɪʏʊeøɘəɵɤoɛœɜɞʌɔæɐaɶɑɒᵻ",                                   # vowels
    "ʘɓǀɗǃʄǂɠǁʛ",                                                     # non-pulmonic consonants
    "pbtdʈɖcɟkɡqɢʔɴŋɲɳnɱmʙrʀⱱɾɽɸβfvθðszʃʒʂʐçʝxɣχʁħʕhɦɬɮʋɹɻjɰlɭʎʟ",  # pulmonic consonants
    "ˈˌːˑ",                                                           # suprasegmentals
    "ʍwɥʜʢʡɕʑɺɧ ",                                                    # other symbols
    "ɚ˞ɫ",                                                            # diacritics
)
PHONEME_CHARS = sorted("".join(_IPA_GROUPS))
SYMBOLS = [PAD, EOS, BOS] + list(CHARACTERS) + ["@" + p for p in PHONEME_CHARS]
PHONEMES = [PAD, EOS, BOS] + PHONEME_CHARS + list(PUNCTUATIONS)

_symbol_to_id = {s: i for i, s in enumerate(SYMBOLS)}
_id_to_symbol = {i: s for i, s in enumerate(SYMBOLS)}
_curly_re = re.compile(r"(.*?)\{(.+?)\}(.*)")
_whitespace_re = re.compile(r"\s+")


def lowercase(text):
    return text.lower()


def collapse_whitespace(text):
    return re.sub(_whitespace_re, " ", text).strip()


def basic_cleaners(text):
    """cleaners.py:66-70: lowercase, collapse whitespace; no transliteration."""
    return collapse_whitespace(lowercase(text))


_CLEANERS = {"basic_cleaners": basic_cleaners}
_NEEDS = {"transliteration_cleaners": "unidecode", "english_cleaners": "unidecode + inflect",
          "phoneme_cleaners": "unidecode + inflect"}


def _clean_text(text, cleaner_names):
    for name in cleaner_names:
        if name not in _CLEANERS:
            if name in _NEEDS:
                raise NotImplementedError(f"cleaner {name!r} needs {_NEEDS[name]}, which is not installed")
            raise Exception("Unknown cleaner: %s" % name)
        text = _CLEANERS[name](text)
    return text


def _keep(s):
    return s in _symbol_to_id and s not in (EOS, BOS, PAD)


def _symbols_to_sequence(symbols):
    return [_symbol_to_id[s] for s in symbols if _keep(s)]


def text_to_sequence(text, cleaner_names):
    """utils/text/__init__.py:77-99: ids of the cleaned text; ``{...}`` spans are ARPAbet."""
    sequence = []
    while len(text):
        m = _curly_re.match(text)
        if not m:
            sequence += _symbols_to_sequence(_clean_text(text, cleaner_names))
            break
        sequence += _symbols_to_sequence(_clean_text(m.group(1), cleaner_names))
        sequence += _symbols_to_sequence(["@" + s for s in m.group(2).split()])
        text = m.group(3)
    return sequence


def sequence_to_text(sequence):
    """utils/text/__init__.py:102-112."""
    result = ""
    for symbol_id in sequence:
        if symbol_id in _id_to_symbol:
            s = _id_to_symbol[symbol_id]
            if len(s) > 1 and s[0] == "@":
                s = "{%s}" % s[1:]
            result += s
    return result.replace("}{", " ")


def phoneme_to_sequence(text, cleaner_names, language, enable_eos_bos=False):
    raise NotImplementedError("phoneme_to_sequence needs phonemizer + espeak, which are not installed")


def num_chars(config):
    """Size of the embedding table the reference builds for a config (synthesize.py:88-89)."""
    return len(PHONEMES) if config.get("use_phonemes", False) else len(SYMBOLS)
