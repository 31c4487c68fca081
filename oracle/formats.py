"""CPU oracle for the record formats (TEST INFRASTRUCTURE ONLY; the product path is
csrc/formats.cpp behind the C-ABI).  Pure-Python restatement of

* ``Double.toString(double)`` -- java.lang.Double javadoc (JDK >= 19 wording): layout
  ``[-]ddd.ddd`` for 1e-3 <= |v| < 1e7, else ``d.dddE[-]n``, at least one fractional digit;
  digits = the shortest decimal that rounds to v (closest on ties), and when one digit
  suffices, the closest decimal of length 1 or 2.  Python's ``repr`` yields the shortest,
  closest digits, so only the layout and the length-2 rule are restated here.
* ``Double.parseDouble`` -- FloatingDecimal.readJavaFormatString's grammar (trim, sign,
  NaN / Infinity / decimal / hex with a binary exponent, optional f/F/d/D suffix).
* ``String.split(" ")`` (trailing empty strings dropped; no match -> the whole string).
* the reference's record code: MapperDataset_github.java:12-20 (dataset lines),
  CreateLocalMST.java:110-123 (local-MST text), UnionFindReducer.java:22-45 (its parse).

Parity pin: the javadoc-stated values (Double.MIN_VALUE = 4.9E-324, MAX_VALUE =
1.7976931348623157E308, 1.0E7, 0.001, 1.0E-4 ...) in tests/test_formats.py.  JDK 8 can print
a longer digit string for rare values (JDK-4511638); those are parity-unpinned (both parse
back to the same double).
"""
from __future__ import annotations

import math
import re

_DEC = re.compile(r"[+-]?(?:NaN|Infinity|(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?[fFdD]?|"
                  r"0[xX](?:[0-9a-fA-F]+\.?[0-9a-fA-F]*|\.[0-9a-fA-F]+)[pP][+-]?\d+[fFdD]?)")


class NumberFormatException(ValueError):
    pass


def java_split(s: str, sep: str = " "):
    parts = s.split(sep)
    if len(parts) == 1:
        return parts
    while parts and parts[-1] == "":
        parts.pop()
    return parts


def parse_double(s: str) -> float:
    t = s.strip("".join(chr(c) for c in range(33)))
    if not _DEC.fullmatch(t):
        raise NumberFormatException(f'For input string: "{s}"')
    body, suffix = t, ""
    if body[-1] in "fFdD":  # hex needs a decimal binary exponent, so a final f/d is a suffix
        suffix, body = body[-1], body[:-1]
    if body.lstrip("+-").lower().startswith("0x"):
        v = float.fromhex(body)
    else:
        v = float(body.replace("Infinity", "inf"))
    # a type suffix does not influence the result (Double.parseDouble javadoc)
    return v


def parse_int(s: str) -> int:
    if not re.fullmatch(r"[+-]?\d+", s):
        raise NumberFormatException(f'For input string: "{s}"')
    v = int(s)
    if not -2**31 <= v < 2**31:
        raise NumberFormatException(f'For input string: "{s}"')
    return v


def double_to_string(v: float) -> str:
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "Infinity" if v > 0 else "-Infinity"
    sign = "-" if math.copysign(1.0, v) < 0 else ""
    v = abs(float(v))
    if v == 0.0:
        return sign + "0.0"
    r = repr(v)                              # shortest, closest digits
    m = re.fullmatch(r"(\d+)(?:\.(\d+))?(?:e([+-]\d+))?", r)
    ip, fp, e = m.group(1), m.group(2) or "", int(m.group(3) or 0)
    digits = (ip + fp).lstrip("0")
    # decimal exponent of the first significant digit
    lead_zeros = len(ip + fp) - len((ip + fp).lstrip("0"))
    E = len(ip) - 1 - lead_zeros + e
    digits = digits.rstrip("0") or "0"
    if len(digits) == 1:  # length-2 rule: the correctly rounded 2-digit decimal
        s2 = f"{v:.1e}"
        digits = (s2[0] + s2[2]).rstrip("0") or "0"
        E = int(s2.split("e")[1])
    if -3 <= E <= 6:
        if E >= 0:
            ipart = (digits + "0" * (E + 1))[: E + 1]
            fpart = digits[E + 1:] or "0"
            return f"{sign}{ipart}.{fpart}"
        return f"{sign}0.{'0' * (-E - 1)}{digits}"
    return f"{sign}{digits[0]}.{digits[1:] or '0'}E{E}"


def dataset_line(s: str, d: int = 0, strict: bool = True):
    """MapperDataset_github.call's point (strict) or the D1 reading (whitespace, first d)."""
    fields = java_split(s, " ") if strict else [f for f in re.split(r"[ \t]+", s) if f]
    if not strict and d:
        fields = fields[:d]
    return [parse_double(f) for f in fields]


def read_dataset(text: str, d: int = 0, strict: bool = True):
    rows = []
    lines = text.split("\n")
    if lines and lines[-1] == "":
        lines.pop()  # a final newline ends the last record
    for ln in lines:
        ln = ln[:-1] if ln.endswith("\r") else ln
        if not strict and not ln.strip(" \t"):
            continue
        rows.append(dataset_line(ln, d, strict))
    return rows


def format_local_mst(va, vb, w, fake1=None, fake2=None, node=None) -> str:
    n = len(va)
    z = [0] * n
    fake1, fake2, node = (z if a is None else a for a in (fake1, fake2, node))
    return "\n".join(f"{int(va[i])} {int(vb[i])} {double_to_string(float(w[i]))} {int(fake1[i])} "
                     f"{int(fake2[i])} {int(node[i])}" for i in range(n))


def parse_local_mst(text: str):
    out = []
    for ln in java_split(text, "\n"):
        data = java_split(ln, " ")
        rec = []
        for k in range(6):  # UnionFindReducer.java:26-31: data[0..5] parsed in order
            if k >= len(data):
                raise IndexError(len(data))
            rec.append(parse_double(data[k]) if k == 2 else parse_int(data[k]))
        out.append(tuple(rec))
    return out
