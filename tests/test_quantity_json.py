"""Quantity semantics (k8s.io/apimachinery resource.Quantity) and the JSON DOM."""
import json

import pytest

from flex_gpu_scheduler_amd._native import native

X = native()


@pytest.mark.parametrize("s,milli,value,canon", [
    ("1", 1000, 1, "1"),
    ("500m", 500, 1, "500m"),
    ("1.5", 1500, 2, "1500m"),
    ("2k", 2000000, 2000, "2k"),
    ("1500", 1500000, 1500, "1500"),
    ("1Gi", 1073741824000, 1073741824, "1Gi"),
    ("1536Mi", 1610612736000, 1610612736, "1536Mi"),
    ("2048Mi", 2147483648000, 2147483648, "2Gi"),
    ("1e3", 1000000, 1000, "1e3"),
    ("100n", 1, 1, "100n"),
    ("0.1", 100, 1, "100m"),
    ("288", 288000, 288, "288"),
    ("0", 0, 0, "0"),
])
def test_quantity_parse(s, milli, value, canon):
    m, v, c = X.parse_quantity(s)
    assert (m, v, c) == (milli, value, canon)


@pytest.mark.parametrize("bad", ["", "abc", "1.2.3", "5Xi", "--1", "1e"])
def test_quantity_rejects(bad):
    with pytest.raises(Exception):
        X.parse_quantity(bad)


def test_json_roundtrip_unicode_and_numbers():
    doc = {"a": [1, -2, 3.5, True, None, "x\"y\né"], "b": {"c": {}}, "big": 9007199254740993}
    out = json.loads(X.json_roundtrip(json.dumps(doc)))
    assert out == doc


def test_merge_patch_rfc7386():
    a = {"a": "b", "c": {"d": "e", "f": "g"}}
    assert X.merge_patch(a, {"a": "z", "c": {"f": None}}) == {"a": "z", "c": {"d": "e"}}
    assert X.merge_patch({"a": [1, 2]}, {"a": [3]}) == {"a": [3]}
    assert X.merge_patch({"a": 1}, {"b": {"c": None}}) == {"a": 1, "b": {}}


def test_rfc3339_roundtrip():
    us = 1_700_000_000_123_456
    assert X.parse_rfc3339(X.rfc3339(us)) == us
    assert X.parse_rfc3339("2024-02-29T12:00:00Z") == 1709208000 * 1_000_000
    assert X.parse_rfc3339("2024-02-29T13:00:00+01:00") == 1709208000 * 1_000_000
