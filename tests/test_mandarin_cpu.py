"""Mandarin synthesis frontend: pinyin -> phones through the shipped lexicon (reference
``synthesize.py:65-90``, ``lexicon/pinyin-lexicon-r.txt``), checked against the AISHELL3 ``val.txt``
fixture (pinyin column vs MFA phone column).  Hanzi -> pinyin is parity-unpinned (no fixture) and is
rejected instead of synthesised as silence."""
import os
import re
from collections import defaultdict

import pytest

from speakingstyle_amd.text import g2p, text_to_sequence

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LEX = os.path.join(ROOT, "lexicon", "pinyin-lexicon-r.txt")
VAL = "/root/reference/preprocessed_data/AISHELL3/val.txt"


def _alternatives():
    alts = defaultdict(list)
    for line in open(LEX, encoding="utf-8"):
        parts = line.split()
        if len(parts) >= 2:
            alts[parts[0].lower()].append(parts[1:])
    return alts


def test_lexicon_shipped_and_first_entry_wins():
    lex = g2p.load_lexicon("lexicon/pinyin-lexicon-r.txt", "zh")
    assert len(lex) > 4000 - 100
    # duplicate keys (er1..er5 -> 'erN' and 'eN rr'): the first entry wins, as in the reference's read_lexicon
    assert lex["er4"] == ["er4"]
    assert lex["ni3"] == ["n", "i3"]


@pytest.mark.skipif(not os.path.exists(VAL), reason="reference AISHELL3 val.txt fixture not present")
def test_val_pinyin_maps_to_phones():
    lex = g2p.load_lexicon(LEX, "zh")
    alts = _alternatives()
    n = 0
    for line in open(VAL, encoding="utf-8"):
        base, spk, phones, pinyin = line.rstrip("\n").split("|")
        want = [p for p in phones.strip("{}").split() if p != "sp"]
        syl = pinyin.split()
        got = [p for p in g2p.mandarin_phones(syl, lex) if p != "sp"]
        # MFA aligned with the lexicon's second 'er' spelling ('e4 rr'); the reference's synthesis (first
        # entry) says 'er4'.  Every syllable must match one of its lexicon entries, in order.
        pos = 0
        for s in syl:
            for cand in alts[s]:
                if want[pos:pos + len(cand)] == cand:
                    pos += len(cand)
                    break
            else:
                raise AssertionError(f"{base}: syllable {s} does not match {want[pos:pos + 3]}")
        assert pos == len(want), base
        assert len(got) == sum(len(alts[s][0]) for s in syl)
        # every phone is in the symbol set (no '@' lookups dropped)
        seq = text_to_sequence("{" + " ".join(got) + "}", [])
        assert len(seq) == len(got), base
        n += 1
    assert n == 512


def test_missing_lexicon_and_hanzi_fail_loudly(tmp_path):
    with pytest.raises(FileNotFoundError):
        g2p.load_lexicon(str(tmp_path / "none.txt"), "zh")
    assert g2p.load_lexicon(str(tmp_path / "none.txt"), "en") == {}
    with pytest.raises(ValueError):
        g2p.preprocess_mandarin(["ni3"], [], {})
    lex = g2p.load_lexicon(LEX, "zh")
    with pytest.raises(ValueError):
        g2p.preprocess_mandarin(["你好"], [], lex)
    with pytest.warns(UserWarning):
        _, ph = g2p.preprocess_mandarin(["ni3", "xyz9", "qqq1", "，"], [], lex)
    assert ph == ["n", "i3", "sp", "sp", "sp"]


def test_single_batch_zh_not_silence():
    from speakingstyle_amd.config import load_named
    from speakingstyle_amd.infer.synthesis import single_batch

    pp, mc, tc = load_named("AISHELL3")
    lex = g2p.load_lexicon(pp["path"]["lexicon_path"], "zh")
    batch, phones, _ = single_batch("ni3 hao3 shi4 jie4", pp, 0, None, lex)
    assert phones == ["n", "i3", "h", "ao3", "sh", "iii4", "j", "ie4"]
    assert all(re.fullmatch(r"[a-z]+\d?", p) and p != "sp" for p in phones)
