"""Kubernetes resource.Quantity parsing (the subset the scheduler needs).

Semantics follow k8s.io/apimachinery/pkg/api/resource: decimal SI suffixes
(k, M, G, T, P, E, and m for milli), binary suffixes (Ki ... Ei) and decimal
exponents (1e3).  ``as_int64`` mirrors ``Quantity.AsInt64()``: it only
succeeds for values that are exact integers; ``value`` mirrors
``Quantity.Value()`` (rounds up to an integer).
"""

from __future__ import annotations

import math
from decimal import Decimal, InvalidOperation

_BIN = {"Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_DEC = {"n": Decimal("1e-9"), "u": Decimal("1e-6"), "m": Decimal("1e-3"), "": Decimal(1),
        "k": Decimal(10) ** 3, "M": Decimal(10) ** 6, "G": Decimal(10) ** 9, "T": Decimal(10) ** 12,
        "P": Decimal(10) ** 15, "E": Decimal(10) ** 18}


class QuantityError(ValueError):
    pass


def parse(q) -> Decimal:
    if isinstance(q, bool):
        raise QuantityError(f"invalid quantity {q!r}")
    if isinstance(q, (int,)):
        return Decimal(q)
    if isinstance(q, float):
        return Decimal(str(q))
    if isinstance(q, Decimal):
        return q
    s = str(q).strip()
    if not s:
        raise QuantityError("empty quantity")
    for suf, mult in _BIN.items():
        if s.endswith(suf):
            return _num(s[: -len(suf)]) * mult
    if s[-1].isalpha():
        if s[-1] not in _DEC:
            raise QuantityError(f"invalid quantity suffix in {q!r}")
        return _num(s[:-1]) * _DEC[s[-1]]
    return _num(s)


def _num(s: str) -> Decimal:
    # Decimal() also takes "1_000", " 1" (as in "1 Gi"), "Infinity" and "NaN";
    # a Quantity takes none of them
    if "_" in s or any(c.isspace() for c in s):
        raise QuantityError(f"invalid quantity number {s!r}")
    try:
        d = Decimal(s)
    except InvalidOperation as e:
        raise QuantityError(f"invalid quantity number {s!r}") from e
    if not d.is_finite():
        raise QuantityError(f"invalid quantity number {s!r}")
    return d


def as_int64(q) -> tuple[int, bool]:
    """(value, ok): ok only when q is an exact integer within int64."""
    try:
        d = parse(q)
    except QuantityError:
        return 0, False
    if d != d.to_integral_value():
        return 0, False
    v = int(d)
    if v < -(2 ** 63) or v >= 2 ** 63:
        return 0, False
    return v, True


def value(q) -> int:
    """Quantity.Value(): ceil to integer."""
    d = parse(q)
    return int(math.ceil(d))
