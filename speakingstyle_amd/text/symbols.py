"""Model input symbol table.

Index order is part of the checkpoint contract: the phoneme embedding
``encoder.src_word_emb`` is indexed by these ids, so the table reproduces the
reference ordering (``text/symbols.py:10-29`` of the reference): pad, '-',
punctuation, ASCII letters, '@'-prefixed ARPAbet (84), '@'-prefixed pinyin (209),
'@' silences (3) -> 360 symbols; the embedding has len(symbols)+1 = 361 rows.
The ARPAbet / pinyin inventories are generated rather than listed.
"""

PAD = "_"
SPECIAL = "-"
PUNCTUATION = "!'(),.:;? "
LETTERS = "".join(chr(c) for c in range(ord("A"), ord("Z") + 1)) + "".join(
    chr(c) for c in range(ord("a"), ord("z") + 1)
)
SILENCES = ["@sp", "@spn", "@sil"]

# CMUdict ARPAbet: vowels carry a stress-less form plus stresses 0..2
_ARPA_VOWELS = ["AA", "AE", "AH", "AO", "AW", "AY", "EH", "ER", "EY", "IH", "IY", "OW", "OY", "UH", "UW"]
_ARPA_CONSONANTS = ["B", "CH", "D", "DH", "F", "G", "HH", "JH", "K", "L", "M", "N", "NG",
                    "P", "R", "S", "SH", "T", "TH", "V", "W", "Y", "Z", "ZH"]


def _arpabet():
    out = []
    for p in _ARPA_VOWELS:
        out += [p] + [p + str(s) for s in range(3)]
    out += _ARPA_CONSONANTS
    return sorted(out)


ARPABET = _arpabet()

PINYIN_INITIALS = ["b", "c", "ch", "d", "f", "g", "h", "j", "k", "l", "m", "n", "p", "q",
                   "r", "s", "sh", "t", "w", "x", "y", "z", "zh"]
_PINYIN_FINAL_STEMS = ["a", "ai", "an", "ang", "ao", "e", "ei", "en", "eng", "er", "i", "ia",
                       "ian", "iang", "iao", "ie", "ii", "iii", "in", "ing", "iong", "iou", "o",
                       "ong", "ou", "u", "ua", "uai", "uan", "uang", "uei", "uen", "uo", "v",
                       "van", "ve", "vn"]
PINYIN_FINALS = [f + str(t) for f in _PINYIN_FINAL_STEMS for t in range(1, 6)]
PINYIN = PINYIN_INITIALS + PINYIN_FINALS + ["rr"]

symbols = (
    [PAD]
    + list(SPECIAL)
    + list(PUNCTUATION)
    + list(LETTERS)
    + ["@" + s for s in ARPABET]
    + ["@" + s for s in PINYIN]
    + SILENCES
)

assert len(ARPABET) == 84 and len(PINYIN) == 209 and len(symbols) == 360
