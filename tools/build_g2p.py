#!/usr/bin/env python
"""Learn the in-tree English letter-to-sound model (``speakingstyle_amd/text/lts.py``) from the
LJSpeech metadata shipped with the reference: ``preprocessed_data/LJSpeech/train.txt`` lines
``id|speaker|{MFA ARPAbet phones}|normalized text``.

1. Utterances without ``spn`` (MFA's unknown-word token); pause tokens ``sp`` dropped.  Words =
   ``[a-z']+`` runs of the text.
2. EM over a monotonic alignment of the utterance's letters to its phones: every letter emits
   nothing, one phone or two phones; word boundaries emit nothing, so the Viterbi path splits the
   phone string into words.  Emission probabilities P(e | letter) are re-estimated from the
   forward-backward posteriors (a uniform start, two-phone emissions penalised).
3. Lexicon = most frequent phone string per word over the aligned corpus.
4. Rules = for every context level of ``lts.LEVELS`` the majority emission of a letter in that
   context, kept when seen >= ``--min-count`` times and different from the prediction of the
   more general levels (a decision list with back-off).

Writes ``speakingstyle_amd/text/data/{lj_lexicon.tsv,lts_rules.tsv}`` and prints the phone error
rate on ``val.txt`` (rules only and lexicon + rules).
Usage: python tools/build_g2p.py [--em-utts 3000] [--iters 8] [--min-count 2]"""
import argparse
import collections
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from speakingstyle_amd.text import lts  # noqa: E402

_WORD = re.compile(r"[a-z']+")


def read_corpus(path):
    out = []
    with open(path, encoding="utf-8") as f:
        for line in f:
            parts = line.rstrip("\n").split("|")
            if len(parts) < 4:
                continue
            ph = re.search(r"\{(.*)\}", parts[2]).group(1).split()
            words = _WORD.findall(parts[3].lower())
            out.append((words, ph))
    return out


class Aligner:
    def __init__(self, phones, letters):
        self.P = {p: i for i, p in enumerate(phones)}
        self.L = {c: i for i, c in enumerate(letters)}
        nP, nL = len(phones), len(letters)
        self.nP = nP
        self.e0 = np.full(nL, 0.2)
        self.e1 = np.full((nL, nP), 0.6 / nP)
        self.e2 = np.full((nL, nP * nP), 0.2 / (nP * nP))

    def _tables(self, letters, ph):
        li = np.array([self.L[c] for c in letters])
        pi = np.array([self.P[p] for p in ph])
        e0 = self.e0[li]                                  # [n]
        e1 = self.e1[li][:, pi]                           # [n, m] emission of phone j
        pair = np.zeros(len(ph), dtype=np.int64)
        pair[1:] = pi[:-1] * self.nP + pi[1:]
        e2 = self.e2[li][:, pair]                         # [n, m] emission of phones (j-1, j)
        e2[:, 0] = 0.0
        return li, pi, pair, e0, e1, e2

    def forward_backward(self, letters, ph):
        n, m = len(letters), len(ph)
        li, pi, pair, e0, e1, e2 = self._tables(letters, ph)
        alpha = np.zeros((n + 1, m + 1))
        scale = np.zeros(n + 1)
        alpha[0, 0] = 1.0
        scale[0] = 1.0
        for i in range(1, n + 1):
            a = alpha[i - 1] * e0[i - 1]
            a[1:] += alpha[i - 1, :-1] * e1[i - 1]
            a[2:] += alpha[i - 1, :-2] * e2[i - 1, 1:]
            s = a.sum()
            if s <= 0:
                return None
            alpha[i] = a / s
            scale[i] = s
        if alpha[n, m] <= 0:
            return None
        beta = np.zeros((n + 1, m + 1))
        beta[n, m] = 1.0
        for i in range(n, 0, -1):
            b = beta[i] * e0[i - 1]
            b[:-1] += beta[i, 1:] * e1[i - 1]
            b[:-2] += beta[i, 2:] * e2[i - 1, 1:]
            beta[i - 1] = b / scale[i]
        Z = alpha[n, m]
        # posteriors of each emission at (letter i, ending phone j)
        c0 = (alpha[:-1] * beta[1:] * e0[:, None] / Z).sum(1)
        c1 = alpha[:-1, :-1] * beta[1:, 1:] * e1 / Z
        c2 = alpha[:-1, :-2] * beta[1:, 2:] * e2[:, 1:] / Z
        return li, pi, pair, c0, c1, c2

    def em(self, corpus, iters):
        for it in range(iters):
            n0 = np.zeros_like(self.e0)
            n1 = np.zeros_like(self.e1)
            n2 = np.zeros_like(self.e2)
            used = 0
            for letters, ph in corpus:
                r = self.forward_backward(letters, ph)
                if r is None:
                    continue
                li, pi, pair, c0, c1, c2 = r
                np.add.at(n0, li, c0)
                np.add.at(n1, (li[:, None], pi[None, :]), c1)
                np.add.at(n2, (li[:, None], pair[None, 1:]), c2)
                used += 1
            tot = n0 + n1.sum(1) + n2.sum(1) + 1e-12
            self.e0 = n0 / tot + 1e-6
            self.e1 = n1 / tot[:, None] + 1e-8
            self.e2 = n2 / tot[:, None] * 0.5 + 1e-10  # two-phone emissions stay a little penalised
            print(f"EM iter {it}: {used} utterances", flush=True)

    def viterbi(self, letters, ph):
        n, m = len(letters), len(ph)
        li, pi, pair, e0, e1, e2 = self._tables(letters, ph)
        with np.errstate(divide="ignore"):
            l0, l1, l2 = np.log(e0), np.log(e1), np.log(e2)
        dp = np.full((n + 1, m + 1), -np.inf)
        bp = np.zeros((n + 1, m + 1), dtype=np.int8)
        dp[0, 0] = 0.0
        for i in range(1, n + 1):
            cand0 = dp[i - 1] + l0[i - 1]
            cand1 = np.full(m + 1, -np.inf)
            cand1[1:] = dp[i - 1, :-1] + l1[i - 1]
            cand2 = np.full(m + 1, -np.inf)
            cand2[2:] = dp[i - 1, :-2] + l2[i - 1, 1:]
            stack = np.stack([cand0, cand1, cand2])
            bp[i] = stack.argmax(0)
            dp[i] = stack.max(0)
        if not np.isfinite(dp[n, m]):
            return None
        emits = [None] * n
        j = m
        for i in range(n, 0, -1):
            k = int(bp[i, j])
            emits[i - 1] = ph[j - k:j]
            j -= k
        return emits


def utterance_letters(words):
    letters, owner = [], []
    for wi, w in enumerate(words):
        for c in w:
            letters.append(c)
            owner.append(wi)
    return letters, owner


def edit_distance(a, b):
    prev = list(range(len(b) + 1))
    for i, x in enumerate(a, 1):
        cur = [i] + [0] * len(b)
        for j, y in enumerate(b, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (x != y))
        prev = cur
    return prev[-1]


def per(corpus, predict, strip_stress=False):
    err = tot = 0
    for words, ph in corpus:
        ref = [p for p in ph if p != "sp"]
        hyp = [p for w in words for p in predict(w)]
        if strip_stress:
            ref = [re.sub(r"\d", "", p) for p in ref]
            hyp = [re.sub(r"\d", "", p) for p in hyp]
        err += edit_distance(hyp, ref)
        tot += len(ref)
    return err / max(tot, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--train", default=os.path.join(ROOT, "preprocessed_data", "LJSpeech", "train.txt"))
    ap.add_argument("--val", default=os.path.join(ROOT, "preprocessed_data", "LJSpeech", "val.txt"))
    ap.add_argument("--em-utts", type=int, default=3000)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--min-count", type=int, default=2)
    ap.add_argument("--out", default=os.path.join(ROOT, "speakingstyle_amd", "text", "data"))
    a = ap.parse_args()

    train = [(w, [p for p in ph if p != "sp"]) for w, ph in read_corpus(a.train) if "spn" not in ph]
    val = [(w, ph) for w, ph in read_corpus(a.val) if "spn" not in ph]
    phones = sorted({p for _, ph in train for p in ph})
    letters = sorted({c for w, _ in train for word in w for c in word})
    al = Aligner(phones, letters)
    rng = np.random.default_rng(0)
    sub = [train[i] for i in rng.permutation(len(train))[:a.em_utts]]
    al.em([(utterance_letters(w)[0], ph) for w, ph in sub], a.iters)

    # Viterbi over the whole training set -> per-word pronunciations and per-letter emissions
    lex_counts = collections.defaultdict(collections.Counter)
    ctx = [collections.defaultdict(collections.Counter) for _ in lts.LEVELS]
    aligned = 0
    for words, ph in train:
        ls, owner = utterance_letters(words)
        emits = al.viterbi(ls, ph)
        if emits is None:
            continue
        aligned += 1
        per_word = [[] for _ in words]
        for k, e in enumerate(emits):
            per_word[owner[k]].extend(e)
        for w, p in zip(words, per_word):
            lex_counts[w][" ".join(p)] += 1
        pos = 0
        for w in words:
            for i in range(len(w)):
                e = emits[pos + i]
                out = "_".join(e) if e else lts.EPS
                for lvl, (nl, nr) in enumerate(lts.LEVELS):
                    ctx[lvl][lts.context_key(w, i, nl, nr)][out] += 1
            pos += len(w)
    print(f"aligned {aligned}/{len(train)} training utterances", flush=True)

    lexicon = {w: c.most_common(1)[0][0] for w, c in lex_counts.items()}
    # decision list: general levels first, a specific rule only where it changes the prediction
    rules = {}
    for lvl in range(len(lts.LEVELS) - 1, -1, -1):
        for key, cnt in ctx[lvl].items():
            out, n = cnt.most_common(1)[0]
            if lvl != len(lts.LEVELS) - 1 and n < a.min_count:
                continue
            left, letter, right = key.split("|")
            # what the more general levels predict for this context
            prev = None
            for lvl2 in range(lvl + 1, len(lts.LEVELS)):
                nl, nr = lts.LEVELS[lvl2]
                k2 = f"{left[len(left) - nl:] if nl else ''}|{letter}|{right[:nr]}"
                if k2 in rules:
                    prev = rules[k2]
                    break
            if out != prev:
                rules[key] = out
    os.makedirs(a.out, exist_ok=True)
    with open(os.path.join(a.out, "lj_lexicon.tsv"), "w", encoding="utf-8") as f:
        for w in sorted(lexicon):
            f.write(f"{w}\t{lexicon[w]}\n")
    with open(os.path.join(a.out, "lts_rules.tsv"), "w", encoding="utf-8") as f:
        f.write("# left|letter|right<TAB>emission (phones joined by _, - = none); tools/build_g2p.py\n")
        for k in sorted(rules):
            f.write(f"{k}\t{rules[k]}\n")
    print(f"lexicon {len(lexicon)} words, {len(rules)} rules", flush=True)

    def rules_only(w):
        return lts.word_to_phones(w, rules)

    def lex_rules(w):
        return lexicon[w].split() if w in lexicon else lts.word_to_phones(w, rules)

    # word-level references for the val words the lexicon has never seen (Viterbi split of val)
    oov_err = oov_tot = 0
    for words, ph in val:
        ls, owner = utterance_letters(words)
        emits = al.viterbi(ls, [p for p in ph if p != "sp"])
        if emits is None:
            continue
        per_word = [[] for _ in words]
        for k, e in enumerate(emits):
            per_word[owner[k]].extend(e)
        for w, ref in zip(words, per_word):
            if w not in lexicon:
                oov_err += edit_distance(lts.word_to_phones(w, rules), ref)
                oov_tot += len(ref)
    print(f"PER of the rules on val words outside the induced lexicon: {oov_err / max(oov_tot, 1):.4f} "
          f"({oov_tot} phones)")
    oov = sum(1 for words, _ in val for w in words if w not in lexicon)
    nw = sum(len(words) for words, _ in val)
    print(f"val: {len(val)} utterances, {nw} words, {oov} not in the induced lexicon")
    for name, fn in (("rules only", rules_only), ("lexicon + rules", lex_rules)):
        print(f"PER {name}: {per(val, fn):.4f} (stress ignored: {per(val, fn, strip_stress=True):.4f})")


if __name__ == "__main__":
    main()
