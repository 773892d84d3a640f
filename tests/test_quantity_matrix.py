"""resource.Quantity parsing tables (k8s/quantity.py; semantics of
k8s.io/apimachinery/pkg/api/resource as used by the reference's quota and
request extraction, pkg/device/quota.go, pkg/device/nvidia/device.go)."""

from decimal import Decimal

import pytest
from hypothesis import given, strategies as st

from k8s_vgpu_scheduler_amd.k8s import quantity as Q


@pytest.mark.parametrize("q,want", [
    ("36864", 36864), ("1Ki", 1024), ("1Mi", 1 << 20), ("2Gi", 2 << 30), ("1Ti", 1 << 40), ("1Pi", 1 << 50),
    ("1k", 1000), ("5M", 5 * 10 ** 6), ("3G", 3 * 10 ** 9), ("1T", 10 ** 12), ("1P", 10 ** 15), ("2E", 2 * 10 ** 18),
    ("1e3", 1000), ("1.5Gi", 3 << 29), ("2000m", 2), (" 7 ", 7), ("+4", 4), ("-3", -3), (12, 12), ("0", 0),
])
def test_as_int64_exact(q, want):
    assert Q.as_int64(q) == (want, True)


@pytest.mark.parametrize("q", ["500m", "1.5", "1u", "1n", "0.5k" + "m"])
def test_as_int64_fractional_is_not_ok(q):
    assert Q.as_int64(q) == (0, False)


@pytest.mark.parametrize("q", ["", "junk", "1x", "Mi", "1e", "NaN", "Infinity", "1_000", "1 Gi", True])
def test_invalid(q):
    assert Q.as_int64(q) == (0, False)
    with pytest.raises(Q.QuantityError):
        Q.parse(q)


def test_int64_range():
    assert Q.as_int64("8Ei") == (0, False)            # 2**63: out of range
    assert Q.as_int64(str(2 ** 63 - 1)) == (2 ** 63 - 1, True)
    assert Q.as_int64(str(-(2 ** 63))) == (-(2 ** 63), True)


@pytest.mark.parametrize("q,want", [("500m", 1), ("1", 1), ("1001m", 2), ("1.2", 2), ("-0.5", 0), ("1Ki", 1024)])
def test_value_rounds_up(q, want):
    assert Q.value(q) == want


def test_float_and_decimal_inputs():
    assert Q.parse(0.25) == Decimal("0.25")
    assert Q.parse(Decimal("3")) == 3


@given(st.integers(0, 2 ** 40), st.sampled_from(["", "k", "M", "Ki", "Mi", "Gi"]))
def test_integer_with_suffix_round_trip(n, suf):
    mult = {"": 1, "k": 1000, "M": 10 ** 6, "Ki": 1 << 10, "Mi": 1 << 20, "Gi": 1 << 30}[suf]
    v, ok = Q.as_int64(f"{n}{suf}")
    assert ok == (n * mult < 2 ** 63)
    if ok:
        assert v == n * mult
