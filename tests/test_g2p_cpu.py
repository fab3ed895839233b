"""English grapheme-to-phoneme without g2p_en (reference ``synthesize.py:38-62``): the induced
lexicon + learned letter-to-sound rules of ``text/lts.py`` (``tools/build_g2p.py``) measured on the
LJSpeech metadata shipped with the reference (``preprocessed_data/LJSpeech/val.txt``: normalized
text + MFA phones; utterances with MFA's unknown-word token ``spn`` excluded, pauses ``sp`` ignored).

Measured when the model was built: PER 4.4 % (lexicon + rules), 5.1 % (rules alone), 15.9 % on the
val words that never occur in train.txt; the old letter-name spelling is the baseline it replaces."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAL = os.path.join(ROOT, "preprocessed_data", "LJSpeech", "val.txt")


def _val():
    out = []
    with open(VAL, encoding="utf-8") as f:
        for line in f:
            parts = line.rstrip("\n").split("|")
            ph = re.search(r"\{(.*)\}", parts[2]).group(1).split()
            if "spn" in ph:
                continue
            out.append((re.findall(r"[a-z']+", parts[3].lower()), [p for p in ph if p != "sp"]))
    return out


def _ed(a, b):
    prev = list(range(len(b) + 1))
    for i, x in enumerate(a, 1):
        cur = [i] + [0] * len(b)
        for j, y in enumerate(b, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (x != y))
        prev = cur
    return prev[-1]


def _per(data, fn):
    err = tot = 0
    for words, ref in data:
        hyp = [p for w in words for p in fn(w)]
        err += _ed(hyp, ref)
        tot += len(ref)
    return err / tot


def test_g2p_phone_error_rate_on_ljspeech_val():
    from speakingstyle_amd.text import g2p, lts

    assert lts.available(), "learned LTS rules missing (tools/build_g2p.py)"
    data = _val()[:200]
    per_full = _per(data, lambda w: g2p.english_word_phones(w, {}))
    per_rules = _per(data, lambda w: lts.word_to_phones(w))
    per_spell = _per(data, g2p.spell)
    print(f"PER lexicon+rules {per_full:.4f}, rules only {per_rules:.4f}, letter names {per_spell:.4f}")
    assert per_full <= 0.06
    assert per_rules <= 0.07
    assert per_spell > 0.5  # the replaced fallback


def test_unseen_words_and_pipeline():
    from speakingstyle_amd.text import g2p, lts

    # words absent from the LJSpeech corpus go through the context rules
    assert "tokenizer" not in lts.load_lexicon()
    ph = g2p.english_word_phones("tokenizer", {})
    assert ph[:2] == ["T", "OW1"] and ph[-1].startswith("ER")
    assert g2p.english_word_phones("cnn", {}) == g2p.spell("cnn")  # no vowel letter: letter names
    assert g2p.english_word_phones("hello", {"hello": ["X"]}) == ["X"]  # configured lexicon first
    seq, phones = g2p.preprocess_english("Hello, world!", ["english_cleaners"])
    assert phones == ["HH", "AH0", "L", "OW1", "sp", "W", "ER1", "L", "D"] or phones[4] == "sp"
    assert len(seq) == len(phones)
