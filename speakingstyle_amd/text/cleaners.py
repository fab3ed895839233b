"""Text cleaners (names match the reference's ``text/cleaners.py`` so YAML
``text_cleaners`` lists keep working).  ASCII transliteration uses Unicode NFKD
decomposition instead of the `unidecode` package (not available offline)."""
import re
import unicodedata

from .numbers import normalize_numbers

_whitespace_re = re.compile(r"\s+")
_ABBREVIATIONS = {
    "mrs": "misess", "mr": "mister", "dr": "doctor", "st": "saint", "co": "company",
    "jr": "junior", "maj": "major", "gen": "general", "drs": "doctors", "rev": "reverend",
    "lt": "lieutenant", "hon": "honorable", "sgt": "sergeant", "capt": "captain",
    "esq": "esquire", "ltd": "limited", "col": "colonel", "ft": "fort",
}
_abbrev_re = re.compile(r"\b(%s)\." % "|".join(sorted(_ABBREVIATIONS, key=len, reverse=True)), re.IGNORECASE)
_TRANSLIT = {"ß": "ss", "æ": "ae", "Æ": "AE", "ø": "o", "Ø": "O", "œ": "oe", "Œ": "OE", "ð": "d",
             "þ": "th", "ł": "l", "Ł": "L", "“": '"', "”": '"', "‘": "'", "’": "'", "–": "-", "—": "-"}


def expand_abbreviations(text):
    return _abbrev_re.sub(lambda m: _ABBREVIATIONS[m.group(1).lower()], text)


def expand_numbers(text):
    return normalize_numbers(text)


def lowercase(text):
    return text.lower()


def collapse_whitespace(text):
    return _whitespace_re.sub(" ", text)


def convert_to_ascii(text):
    text = "".join(_TRANSLIT.get(c, c) for c in text)
    text = unicodedata.normalize("NFKD", text)
    return text.encode("ascii", "ignore").decode("ascii")


def basic_cleaners(text):
    return collapse_whitespace(lowercase(text))


def transliteration_cleaners(text):
    return collapse_whitespace(lowercase(convert_to_ascii(text)))


def english_cleaners(text):
    text = lowercase(convert_to_ascii(text))
    text = expand_abbreviations(expand_numbers(text))
    return collapse_whitespace(text)
