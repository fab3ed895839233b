"""English number normalisation (no `inflect` dependency).

Covers what the reference's ``text/numbers.py`` handles via ``inflect``: thousands
separators, currency ($ / £), decimals, ordinals (1st, 22nd) and plain integers,
with years 1000-2999 read as pairs ("nineteen ninety").
"""
import re

_ONES = ["zero", "one", "two", "three", "four", "five", "six", "seven", "eight", "nine", "ten",
         "eleven", "twelve", "thirteen", "fourteen", "fifteen", "sixteen", "seventeen",
         "eighteen", "nineteen"]
_TENS = ["", "", "twenty", "thirty", "forty", "fifty", "sixty", "seventy", "eighty", "ninety"]
_SCALES = [(10 ** 12, "trillion"), (10 ** 9, "billion"), (10 ** 6, "million"), (1000, "thousand")]
_ORD_EXCEPT = {"one": "first", "two": "second", "three": "third", "five": "fifth", "eight": "eighth",
               "nine": "ninth", "twelve": "twelfth"}


def _below_1000(n: int) -> str:
    parts = []
    if n >= 100:
        parts.append(_ONES[n // 100] + " hundred")
        n %= 100
    if n >= 20:
        t = _TENS[n // 10]
        parts.append(t + ("-" + _ONES[n % 10] if n % 10 else ""))
    elif n > 0 or not parts:
        parts.append(_ONES[n])
    return " ".join(parts)


def number_to_words(n: int) -> str:
    if n < 0:
        return "minus " + number_to_words(-n)
    if n < 1000:
        return _below_1000(n)
    parts = []
    for value, name in _SCALES:
        if n >= value:
            parts.append(_below_1000(n // value) + " " + name)
            n %= value
    if n:
        parts.append(_below_1000(n))
    return ", ".join(parts)


def ordinal_words(n: int) -> str:
    w = number_to_words(n)
    head, sep, last = w.rpartition(" ") if " " in w else ("", "", w)
    pre, dash, tail = last.rpartition("-")
    word = tail
    if word in _ORD_EXCEPT:
        word = _ORD_EXCEPT[word]
    elif word.endswith("y"):
        word = word[:-1] + "ieth"
    else:
        word = word + "th"
    last = pre + dash + word
    return head + sep + last


_comma_number_re = re.compile(r"([0-9][0-9\,]+[0-9])")
_decimal_number_re = re.compile(r"([0-9]+\.[0-9]+)")
_pounds_re = re.compile(r"£([0-9\,]*[0-9]+)")
_dollars_re = re.compile(r"\$([0-9\.\,]*[0-9]+)")
_ordinal_re = re.compile(r"[0-9]+(st|nd|rd|th)")
_number_re = re.compile(r"[0-9]+")


def _dollars(m):
    parts = m.group(1).split(".")
    if len(parts) > 2:
        return m.group(1) + " dollars"
    d = int(parts[0]) if parts[0] else 0
    c = int(parts[1]) if len(parts) > 1 and parts[1] else 0
    out = []
    if d:
        out.append("%s %s" % (d, "dollar" if d == 1 else "dollars"))
    if c:
        out.append("%s %s" % (c, "cent" if c == 1 else "cents"))
    return ", ".join(out) if out else "zero dollars"


def _number(m):
    n = int(m.group(0))
    if 1000 < n < 3000:
        if n == 2000:
            return "two thousand"
        if 2000 < n < 2010:
            return "two thousand " + number_to_words(n % 100)
        if n % 100 == 0:
            return number_to_words(n // 100) + " hundred"
        return number_to_words(n // 100) + " " + ("oh " if n % 100 < 10 else "") + number_to_words(n % 100)
    return number_to_words(n)


def normalize_numbers(text: str) -> str:
    text = re.sub(_comma_number_re, lambda m: m.group(1).replace(",", ""), text)
    text = re.sub(_pounds_re, r"\1 pounds", text)
    text = re.sub(_dollars_re, _dollars, text)
    text = re.sub(_decimal_number_re, lambda m: m.group(1).replace(".", " point "), text)
    text = re.sub(_ordinal_re, lambda m: ordinal_words(int(m.group(0)[:-2])), text)
    text = re.sub(_number_re, _number, text)
    return text
