"""Kubernetes resource.Quantity → int64, exactly as the scheduler reads it.

Follows apimachinery ParseQuantity (vendor/k8s.io/apimachinery/pkg/api/resource/
quantity.go:274-400: sign, digits, optional fraction, binary-SI / decimal-SI /
decimal-exponent suffix, non-zero values rounded up to 1e-9) and ScaledValue
(:695-713: ceil at the requested scale).  Values are kept as exact rationals
(numerator, denominator) so no float ever enters the resource path.
"""
from __future__ import annotations

import math
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


# ---------------------------------------------------------------------------- formatting
# Quantity.String (quantity.go:605-615) → CanonicalizeBytes (:417-454): the format a string was
# parsed with (binary-SI suffix → BinarySI, an 'e' exponent → DecimalExponent, else DecimalSI),
# BinarySI shown as DecimalSI below 1024 or when not an integer; decimal mantissa with its
# exponent moved to a multiple of 3 (amount.go:219-243), base-1024 mantissa (:248-255).
DECIMAL_SI, BINARY_SI, DECIMAL_EXPONENT = "DecimalSI", "BinarySI", "DecimalExponent"
_DEC_SUFFIX = {-9: "n", -6: "u", -3: "m", 0: "", 3: "k", 6: "M", 9: "G", 12: "T", 15: "P", 18: "E"}
_BIN_SUFFIX = {0: "", 1: "Ki", 2: "Mi", 3: "Gi", 4: "Ti", 5: "Pi", 6: "Ei"}


def fmt(q) -> str:
    """The Format a quantity string parses with."""
    if isinstance(q, int):
        return DECIMAL_SI
    m = _NUM.match(str(q))
    rest = str(q)[m.end():] if m else ""
    if rest in ("Ki", "Mi", "Gi", "Ti", "Pi", "Ei"):
        return BINARY_SI
    if _EXP.fullmatch(rest):
        return DECIMAL_EXPONENT
    return DECIMAL_SI


def canonical(v: Fraction, form: str) -> str:
    """The canonical string of value v in format `form` (CanonicalizeBytes)."""
    if v == 0:
        return "0"
    if form == BINARY_SI:
        if -1024 < v < 1024 or v.denominator != 1:
            form = DECIMAL_SI
        else:
            n, e = int(v), 0
            while n % 1024 == 0 and e < 6:
                n //= 1024
                e += 1
            return "%d%s" % (n, _BIN_SUFFIX[e])
    # decimal: v = mantissa * 10^exp with no factor of 10 left in the mantissa
    num, den = v.numerator, v.denominator
    exp = 0
    while den != 1:           # values are multiples of 1e-9 (ParseQuantity rounds up to nano)
        num *= 10
        exp -= 1
        g = math.gcd(num, den)
        num, den = num // g, den // g
    while num % 10 == 0:
        num //= 10
        exp += 1
    while exp % 3:
        num *= 10
        exp -= 1
    if form == DECIMAL_EXPONENT:
        return "%d%s" % (num, "" if exp == 0 else "e%d" % exp)
    if exp in _DEC_SUFFIX:
        return "%d%s" % (num, _DEC_SUFFIX[exp])
    return "%de%d" % (num, exp)
