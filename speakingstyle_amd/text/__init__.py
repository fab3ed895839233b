"""Text frontend: cleaners + symbol ids (reference ``text/__init__.py:15-75``)."""
import re

from . import cleaners
from .symbols import symbols

_symbol_to_id = {s: i for i, s in enumerate(symbols)}
_id_to_symbol = {i: s for i, s in enumerate(symbols)}
_curly_re = re.compile(r"(.*?)\{(.+?)\}(.*)")


def _clean_text(text, cleaner_names):
    for name in cleaner_names:
        fn = getattr(cleaners, name, None)
        if fn is None:
            raise ValueError("Unknown cleaner: %s" % name)
        text = fn(text)
    return text


def _keep(s):
    return s in _symbol_to_id and s not in ("_", "~")


def _symbols_to_sequence(syms):
    return [_symbol_to_id[s] for s in syms if _keep(s)]


def text_to_sequence(text, cleaner_names):
    """Plain text -> ids; ``{PH PH ...}`` spans are ARPAbet/pinyin phonemes."""
    seq = []
    while text:
        m = _curly_re.match(text)
        if m is None:
            seq += _symbols_to_sequence(_clean_text(text, cleaner_names))
            break
        seq += _symbols_to_sequence(_clean_text(m.group(1), cleaner_names))
        seq += _symbols_to_sequence(["@" + p for p in m.group(2).split()])
        text = m.group(3)
    return seq


def sequence_to_text(sequence):
    out = []
    for i in sequence:
        s = _id_to_symbol.get(int(i))
        if s is None:
            continue
        out.append("{%s}" % s[1:] if len(s) > 1 and s[0] == "@" else s)
    return "".join(out).replace("}{", " ")


__all__ = ["text_to_sequence", "sequence_to_text", "symbols"]
