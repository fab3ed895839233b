"""Grapheme-to-phoneme for synthesis (reference ``synthesize.py:26-90``).

The reference uses a lexicon file first and falls back to ``g2p_en`` (English) /
``pypinyin`` (Mandarin).  Neither package is available offline.  English words here go
through, in order: the configured lexicon (``librispeech-lexicon.txt`` when present), the
lexicon induced from the LJSpeech alignments shipped with the reference, and the learned
letter-to-sound context rules (``text/lts.py``; PER 4.4 % on the held-out ``val.txt``
utterances, 15.9 % on words never seen in training, ``tests/test_g2p_cpu.py``).  Words without a
vowel letter (acronyms) are spelled with ARPAbet letter names.

Mandarin takes tone-numbered pinyin syllables (``ni3 hao3``) through the shipped
``lexicon/pinyin-lexicon-r.txt`` (the reference's static data); a missing lexicon is an error, as
in the reference, and non-syllable tokens (punctuation) map to ``sp`` like the reference's fallback.
Hanzi -> pinyin has no in-tree dictionary and no fixture (parity unpinned): Hanzi input is rejected.
"""
import os
import re
import warnings
from string import punctuation

from . import lts, text_to_sequence

_LETTER_NAMES = {
    "a": "EY1", "b": "B IY1", "c": "S IY1", "d": "D IY1", "e": "IY1", "f": "EH1 F", "g": "JH IY1",
    "h": "EY1 CH", "i": "AY1", "j": "JH EY1", "k": "K EY1", "l": "EH1 L", "m": "EH1 M", "n": "EH1 N",
    "o": "OW1", "p": "P IY1", "q": "K Y UW1", "r": "AA1 R", "s": "EH1 S", "t": "T IY1", "u": "Y UW1",
    "v": "V IY1", "w": "D AH1 B AH0 L Y UW0", "x": "EH1 K S", "y": "W AY1", "z": "Z IY1",
}


_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def resolve_lexicon_path(path):
    """``path`` as given (cwd-relative, like the reference), else relative to the repository root."""
    if os.path.exists(path) or os.path.isabs(path):
        return path
    alt = os.path.join(_ROOT, path)
    return alt if os.path.exists(alt) else path


def load_lexicon(path, language="en"):
    """The configured lexicon.  English may run without one (induced lexicon + letter-to-sound rules);
    Mandarin may not: the reference opens it unconditionally (``synthesize.py:66``)."""
    p = resolve_lexicon_path(path)
    if os.path.exists(p):
        return read_lexicon(p)
    if language == "zh":
        raise FileNotFoundError(f"Mandarin synthesis needs the pinyin lexicon: {path} not found")
    return {}


def read_lexicon(path):
    lex = {}
    with open(path, encoding="utf-8") as f:
        for line in f:
            parts = re.split(r"\s+", line.strip())
            if len(parts) < 2:
                continue
            word = parts[0].lower()
            lex.setdefault(word, parts[1:])
    return lex


def spell(word):
    """ARPAbet letter names (acronyms, or no letter-to-sound model)."""
    phones = []
    for ch in word.lower():
        phones += _LETTER_NAMES.get(ch, "").split()
    return phones


def english_word_phones(word, lexicon):
    w = word.lower()
    if w in lexicon:
        return list(lexicon[w])
    induced = lts.load_lexicon()
    if w in induced:
        return list(induced[w])
    if not re.search(r"[aeiouy]", w):  # acronym-like: letter names
        return spell(w)
    phones = lts.word_to_phones(w) if lts.available() else []
    return phones or spell(w)


def english_to_phones(text, lexicon=None):
    """Text -> ARPAbet phones; numbers and abbreviations are expanded first (g2p_en does that
    inside the reference's fallback), punctuation becomes ``sp``."""
    from .cleaners import english_cleaners

    lexicon = lexicon or {}
    text = english_cleaners(text).rstrip(punctuation)
    phones = []
    for w in re.split(r"([,;.\-\?\!\s+])", text):
        if not w or w.isspace():
            continue
        if re.fullmatch(r"[,;.\-\?\!]", w):
            phones.append("sp")
            continue
        phones += english_word_phones(w, lexicon)
    return phones


def word_groups(text, lexicon=None):
    """Per-word phoneme counts (for word-level prosody control, cf. the
    reference notebook ``control.ipynb`` cells 17-23)."""
    lexicon = lexicon or {}
    groups = []
    for w in re.split(r"([,;.\-\?\!\s+])", text.rstrip(punctuation)):
        if not w or w.isspace():
            continue
        if re.fullmatch(r"[,;.\-\?\!]", w):
            groups.append((w, ["sp"]))
        else:
            groups.append((w, english_word_phones(w, lexicon)))
    return groups


def preprocess_english(text, cleaners, lexicon=None):
    phones = english_to_phones(text, lexicon)
    return text_to_sequence("{" + " ".join(phones) + "}", cleaners), phones


_PINYIN = re.compile(r"[a-zü]+[1-5]")


def mandarin_phones(pinyin_syllables, lexicon):
    """Tone-numbered syllables -> phones (reference ``synthesize.py:65-80``).  Tokens that are not a
    syllable (punctuation) become ``sp``; a syllable-shaped token missing from the lexicon also becomes
    ``sp`` as in the reference, with a warning instead of silence."""
    if not lexicon:
        raise ValueError("Mandarin synthesis needs the pinyin lexicon (lexicon/pinyin-lexicon-r.txt)")
    phones, unknown = [], []
    for p in pinyin_syllables:
        if re.search(r"[\u3400-\u9fff]", p):
            raise ValueError(f"Hanzi input {p!r}: pass tone-numbered pinyin syllables (e.g. 'ni3 hao3'); "
                             "Hanzi -> pinyin conversion is not available offline")
        q = p.lower()
        if q in lexicon:
            phones += lexicon[q]
        else:
            if _PINYIN.fullmatch(q):
                unknown.append(p)
            phones.append("sp")
    if unknown:
        warnings.warn(f"pinyin syllables not in the lexicon (spoken as sp): {unknown}")
    return phones


def preprocess_mandarin(pinyin_syllables, cleaners, lexicon=None):
    """``pinyin_syllables``: list like ['ni3', 'hao3'] (pypinyin TONE3 output)."""
    phones = mandarin_phones(pinyin_syllables, lexicon)
    return text_to_sequence("{" + " ".join(phones) + "}", cleaners), phones
