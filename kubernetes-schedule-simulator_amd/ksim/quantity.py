"""Kubernetes resource.Quantity → int64, exactly as the scheduler reads it.

Follows apimachinery ParseQuantity (vendor/k8s.io/apimachinery/pkg/api/resource/
quantity.go:274-400: sign, digits, optional fraction, binary-SI / decimal-SI /
decimal-exponent suffix, non-zero values rounded up to 1e-9) and ScaledValue
(:695-713: ceil at the requested scale).  Values are kept as exact rationals
(numerator, denominator) so no float ever enters the resource path.
"""
from __future__ import annotations

import re
from fractions import Fraction
from functools import lru_cache

_SUFFIX = {
    "Ki": (2, 10), "Mi": (2, 20), "Gi": (2, 30), "Ti": (2, 40), "Pi": (2, 50), "Ei": (2, 60),
    "n": (10, -9), "u": (10, -6), "m": (10, -3), "": (10, 0), "k": (10, 3), "M": (10, 6),
    "G": (10, 9), "T": (10, 12), "P": (10, 15), "E": (10, 18),
}
_NUM = re.compile(r"([+-]?)([0-9]*)(?:\.([0-9]*))?")
_EXP = re.compile(r"[eE]([+-]?[0-9]+)")

INT64_MAX = (1 << 63) - 1


class QuantityError(ValueError):
    pass


@lru_cache(maxsize=65536)
def parse(q) -> Fraction:
    """Exact value of a quantity string (or int)."""
    if isinstance(q, bool):
        raise QuantityError("quantity: bool")
    if isinstance(q, int):
        return Fraction(q)
    s = str(q)
    m = _NUM.match(s)
    if not s or not m or (m.group(2) == "" and not m.group(3)):
        raise QuantityError("quantities must match the regular expression: %r" % s)
    sign, whole, frac = m.group(1), m.group(2), m.group(3) or ""
    rest = s[m.end():]
    if rest in _SUFFIX:
        base, exp = _SUFFIX[rest]
    else:
        e = _EXP.fullmatch(rest)
        if not e:
            raise QuantityError("unable to parse quantity's suffix: %r" % s)
        base, exp = 10, int(e.group(1))
    v = Fraction(int(whole or "0") * 10 ** len(frac) + int(frac or "0"), 10 ** len(frac))
    v *= Fraction(base) ** exp
    scaled = v * 1_000_000_000
    if scaled.denominator != 1:  # round up to the nano scale (away from zero)
        n = -(-scaled.numerator // scaled.denominator)
        v = Fraction(n, 1_000_000_000)
    return -v if sign == "-" else v


def _ceil(v: Fraction) -> int:
    return -(-v.numerator // v.denominator)


def value(q) -> int:
    """Quantity.Value(): ceil(q)."""
    return _ceil(parse(q))


def milli_value(q) -> int:
    """Quantity.MilliValue(): ceil(q * 1000)."""
    return _ceil(parse(q) * 1000)


def positive(q) -> bool:
    return parse(q) > 0
