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

import re
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


_GO_FLOAT = re.compile(r"^[-+]?[0-9]*\.?[0-9]+([eE][-+][0-9]+)?$")   # resolve.go:84
_NULLS = {"", "~", "null", "Null", "NULL"}


def _go_parse_int(s: str):
    """strconv.ParseInt(s, 0, 64) of Go 1.11: value, or None on a syntax error (a magnitude
    >= 2^63 is returned as is: it can never decode into an int32)."""
    neg = s[:1] == "-"
    if s[:1] in "+-" and s:
        s = s[1:]
    if not s:
        return None
    if len(s) > 1 and s[0] == "0" and s[1] in "xX":
        if len(s) < 3:
            return None
        base, digits = 16, s[2:]
    elif s[0] == "0":
        base, digits = 8, s[1:]
    else:
        base, digits = 10, s
    v = 0
    for c in digits:
        d = int(c, 36) if c.isascii() and c.isalnum() else 99
        if d >= base:
            return None
        v = v * base + d
    return -v if neg else v


def yaml_int32(node):
    """An int32 field as yaml.v2 v2.2.2 decodes it (resolve.go:86-196, decode.go:443-465);
    ``node`` is a PyYAML composed node or None.  Raises QuantityError when it is no int32."""
    if node is None or (isinstance(node, yaml.ScalarNode) and node.tag == "tag:yaml.org,2002:null"
                        and node.style is None and node.value in _NULLS):
        return 0
    if not isinstance(node, yaml.ScalarNode):
        raise QuantityError("seconds is not a scalar")
    if node.style is not None:   # quoted: a !!str, which no int field accepts
        raise QuantityError(f"cannot unmarshal !!str `{node.value}` into int32")
    s = node.value
    if s in _NULLS:
        return 0

    def fits(v):
        if not -(1 << 31) <= v < (1 << 31):
            raise QuantityError(f"seconds {s} overflows int32")
        return v

    def from_float(f):
        if not f <= 9223372036854775807.0 or f < -(1 << 63):
            raise QuantityError(f"seconds {s} overflows int32")
        return fits(int(f))   # Go's int64(float64) truncates toward zero

    if s[0] == ".":
        if not re.fullmatch(r"\.[0-9]+([eE][-+]?[0-9]+)?", s):
            raise QuantityError(f"seconds {s} is not a number")
        return from_float(float(s))
    if not (s[0].isdigit() or s[0] in "+-"):
        raise QuantityError(f"seconds {s} is not an int")   # bools, words, .inf ...
    if re.match(r"^[0-9]{4}-", s):
        raise QuantityError(f"seconds {s} is a timestamp")
    plain = s.replace("_", "")
    v = _go_parse_int(plain)
    if v is not None:
        return fits(v)
    if _GO_FLOAT.match(plain):
        return from_float(float(plain))
    for pre, sign in (("0b", 1), ("-0b", -1)):
        if plain.startswith(pre) and plain[len(pre):] and set(plain[len(pre):]) <= {"0", "1"}:
            return fits(sign * int(plain[len(pre):], 2))
    raise QuantityError(f"seconds {s} is not an int")


def _plain(node):
    """literal text of the scalars of a composed node (decode.go:420-428: scalars decode into
    strings as their text), or the node itself when not a mapping/sequence/scalar"""
    if isinstance(node, yaml.MappingNode):
        return {k.value: _plain(v) for k, v in node.value}
    if isinstance(node, yaml.SequenceNode):
        return [_plain(v) for v in node.value]
    return None if (node.style is None and node.value in _NULLS) else node.value


def parse_simspec(text: str):
    root = yaml.compose(text, Loader=yaml.BaseLoader)
    if root is None:
        return []
    if not isinstance(root, yaml.SequenceNode):
        raise QuantityError("simSpec is not a YAML list")
    phases = []
    for item in root.value:
        fields = {k.value: v for k, v in item.value} if isinstance(item, yaml.MappingNode) else {}
        ru = fields.get("resourceUsage")
        if ru is not None and isinstance(ru, yaml.SequenceNode):
            raise QuantityError("resourceUsage is not a mapping")   # yaml.v2 type error
        if ru is None or not isinstance(ru, yaml.MappingNode):
            raise InvalidResourceUsageField("Invalid spec.resoruceUsage field")
        sec = yaml_int32(fields.get("seconds"))
        phases.append((sec, build_resource_list({k: ("" if v is None else v) for k, v in _plain(ru).items()})))
    return phases
