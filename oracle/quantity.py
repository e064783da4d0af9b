"""Restatement of k8s ``resource.ParseQuantity`` and kubesim's simSpec decoding.

TEST INFRASTRUCTURE ONLY (pins the units and ingest rules the traces use).

* ``parse_quantity``: ``vendor/k8s.io/apimachinery/pkg/api/resource/quantity.go:146-380``
  (scanner :146-260, suffixes ``suffix.go`` — "", n u m k M G T P E, Ki Mi Gi Ti Pi Ei,
  e/E exponents; non-zero values round up (away from zero) to the nano scale :350-358;
  BinarySI values are capped at 2^63-1 :363-366).  Returns the exact value as a Fraction.
* ``to_milli``: the engine's unit; ``None`` when the value is not a whole number of
  milli-units (outside the exact int64 domain the device path accepts).
* ``build_resource_list``: ``kubesim/util/util.go:11-23`` (InvalidArgument on a bad value).
* ``parse_simspec``: ``kubesim/pod/spec.go:25-63`` — a YAML list of {seconds: int32,
  resourceUsage: map[name]string}; a missing/null resourceUsage is
  ``errInvalidResourceUsageField`` (:48-50).  yaml.v2 decodes scalars into the string
  map as their literal text (vendor/gopkg.in/yaml.v2/decode.go:420-428); PyYAML's
  BaseLoader keeps literal text too.
"""
from __future__ import annotations

from fractions import Fraction

import yaml

_DEC = {"": 0, "n": -9, "u": -6, "m": -3, "k": 3, "M": 6, "G": 9, "T": 12, "P": 15, "E": 18}
_BIN = {"Ki": 10, "Mi": 20, "Gi": 30, "Ti": 40, "Pi": 50, "Ei": 60}
MAX_INT64 = (1 << 63) - 1


class QuantityError(ValueError):
    pass


class InvalidResourceUsageField(ValueError):
    """errInvalidResourceUsageField (kubesim/pod/spec.go:22)."""


def _split(s: str):
    """parseQuantityString (quantity.go:146-260)."""
    pos, end = 0, len(s)
    positive = True
    if pos < end and s[0] in "+-":
        positive = s[0] == "+"
        pos += 1
    while pos < end and s[pos] == "0":
        pos += 1
    if pos >= end:
        return positive, "0", "", ""
    i = pos
    while i < end and s[i].isdigit():
        i += 1
    num = s[pos:i] or "0"
    pos = i
    denom = ""
    if pos < end and s[pos] == ".":
        pos += 1
        i = pos
        while i < end and s[i].isdigit():
            i += 1
        denom = s[pos:i]
        pos = i
    suf_start = pos
    i = pos
    while i < end and s[i] in "eEinumkKMGTP":
        i += 1
    pos = i
    if pos < end and s[pos] in "+-":
        pos += 1
    while pos < end:
        if not s[pos].isdigit():
            raise QuantityError(f"quantities must match the regular expression: {s!r}")
        pos += 1
    return positive, num, denom, s[suf_start:end]


def parse_quantity(s: str) -> Fraction:
    if len(s) == 0:
        raise QuantityError("empty quantity")
    if s == "0":
        return Fraction(0)
    positive, num, denom, suf = _split(s)
    if suf in _DEC:
        base, exp = 10, _DEC[suf]
    elif suf in _BIN:
        base, exp = 2, _BIN[suf]
    elif len(suf) > 1 and suf[0] in "eE":
        try:
            base, exp = 10, int(suf[1:])
        except ValueError:
            raise QuantityError(f"unable to parse quantity's suffix: {s!r}")
    else:
        raise QuantityError(f"unable to parse quantity's suffix: {s!r}")
    v = Fraction(int(num + denom), 10 ** len(denom)) * Fraction(base) ** exp
    # round non-zero values up (away from zero) to the nano scale
    nano = v * 10 ** 9
    if nano.denominator != 1:
        nano = Fraction(-((-nano.numerator) // nano.denominator))
    v = nano / 10 ** 9
    if base == 2 and v > MAX_INT64:
        v = Fraction(MAX_INT64)
    return v if positive else -v


def to_milli(q: Fraction):
    m = q * 1000
    return int(m) if m.denominator == 1 else None


def value_ceil(q: Fraction) -> int:
    """Quantity.Value(): rounds up (quantity.go:684-686)."""
    return -((-q.numerator) // q.denominator)


def build_resource_list(d: dict) -> dict:
    out = {}
    for k, v in d.items():
        try:
            out[k] = parse_quantity(str(v))
        except QuantityError:
            raise QuantityError(f"invalid {k} value {v!r}")
    return out


def parse_simspec(text: str):
    doc = yaml.load(text, Loader=yaml.BaseLoader)
    if doc is None:
        return []
    phases = []
    for item in doc:
        ru = item.get("resourceUsage") if isinstance(item, dict) else None
        if ru is None or not isinstance(ru, dict):
            raise InvalidResourceUsageField("Invalid spec.resoruceUsage field")
        sec = int(item.get("seconds", "0"))
        if not -(1 << 31) <= sec < (1 << 31):
            raise QuantityError("seconds out of int32 range")
        phases.append((sec, build_resource_list(ru)))
    return phases
