"""Letter-to-sound for English words outside the lexicon (the reference runs ``g2p_en`` there,
``synthesize.py:38-62``; that package -- and ``librispeech-lexicon.txt`` -- are not available).

Two data files learned from the LJSpeech metadata shipped with the reference
(``preprocessed_data/LJSpeech/train.txt``: normalized text + MFA ARPAbet phones) by
``tools/build_g2p.py``:

* ``data/lj_lexicon.tsv`` -- word -> phones, induced by aligning every training utterance's
  letters to its phone string (EM over monotonic letter -> {nothing, one phone, two phones}
  emissions, then the Viterbi path; the word boundaries split the phones);
* ``data/lts_rules.tsv`` -- context rules ``left|letter|right -> emission`` over the same
  alignments: each rule is the majority emission of a letter in that spelling context, kept only
  where it differs from the rule one context level down (a backed-off decision list).  A word is
  converted letter by letter with the longest matching context, ``#`` marking the word edges.

``tests/test_g2p_cpu.py`` measures the phone error rate on the held-out ``val.txt`` utterances.
"""
from __future__ import annotations

import os
from functools import lru_cache
from typing import Dict, List, Tuple

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
LEXICON_FILE = os.path.join(_DATA, "lj_lexicon.tsv")
RULES_FILE = os.path.join(_DATA, "lts_rules.tsv")

# context levels, most specific first: (letters to the left, letters to the right)
LEVELS: Tuple[Tuple[int, int], ...] = ((4, 4), (3, 4), (4, 3), (3, 3), (2, 3), (3, 2), (2, 2), (1, 2), (2, 1),
                                       (1, 1), (0, 2), (2, 0), (0, 1), (1, 0), (0, 0))
EPS = "-"  # the empty emission


def context_key(word: str, i: int, nl: int, nr: int) -> str:
    """``left|letter|right`` around letter ``i`` of ``word`` (``#`` past the word edges)."""
    w = "####" + word + "####"
    j = i + 4
    return f"{w[j - nl:j]}|{w[j]}|{w[j + 1:j + 1 + nr]}"


@lru_cache(maxsize=1)
def load_rules(path: str = RULES_FILE) -> Dict[str, str]:
    rules: Dict[str, str] = {}
    if not os.path.exists(path):
        return rules
    with open(path, encoding="utf-8") as f:
        for line in f:
            line = line.rstrip("\n")
            if not line or line.startswith("# "):  # header; rule keys themselves start with "#"
                continue
            k, v = line.split("\t")
            rules[k] = v
    return rules


@lru_cache(maxsize=1)
def load_lexicon(path: str = LEXICON_FILE) -> Dict[str, List[str]]:
    lex: Dict[str, List[str]] = {}
    if not os.path.exists(path):
        return lex
    with open(path, encoding="utf-8") as f:
        for line in f:
            parts = line.rstrip("\n").split("\t")
            if len(parts) == 2 and parts[1]:
                lex[parts[0]] = parts[1].split()
    return lex


def word_to_phones(word: str, rules: Dict[str, str] = None) -> List[str]:
    """Letter-to-sound of one lower-case word with the learned context rules."""
    rules = load_rules() if rules is None else rules
    out: List[str] = []
    for i in range(len(word)):
        emit = None
        for nl, nr in LEVELS:
            emit = rules.get(context_key(word, i, nl, nr))
            if emit is not None:
                break
        if emit and emit != EPS:
            out.extend(emit.split("_"))
    return out


def available() -> bool:
    return bool(load_rules())
