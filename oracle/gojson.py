"""Test-only restatement of the reference's gossip wire format (SURVEY §8(f)
row 2).  Never imported by crdt_amd.

  * marshal_diff  -- server.Diff.ToJSON() as served by the Gossip handler
    (main.go:153-170, :159): gods v1.18.1 treemap ToJSON builds
    map[string]interface{}{strconv.FormatInt(ts): value} and json.Marshal's
    it (Go 1.18 encoding/json): map keys sorted as byte strings, no spaces,
    strings escaped HTML-safe (\\u003c \\u003e \\u0026), \\n \\r \\t kept
    short, other bytes < 0x20 as \\u00xx, U+2028/U+2029 escaped, each byte of
    invalid UTF-8 as \\ufffd.
  * ingest        -- the gossip pull (main.go:245-256): json.Unmarshal into
    map[string]map[string]string (error: round skipped, outcome 1), then
    RemoteDiff.Put(int64(Atoi(key)), value) per key; a failed Atoi ends the
    goroutine (outcome 2, nothing ingested -- "that key first" is one of Go's
    random map orders).  Keys with equal Atoi values are applied in byte
    order of the key strings, the last winning.  For valid UTF-8 input only
    (invalid-byte cases are pinned by the hand-written KATs instead).

Values are Python dicts (str -> str); Diff values that are local writes
(*Command, main.go:187) marshal exactly like remote maps.
"""
from __future__ import annotations

import json
from typing import Dict, Tuple

_HEX = "0123456789abcdef"


def _utf8_decode_rune(b: bytes, i: int):
    """(code point or None, length) like Go's utf8.DecodeRune."""
    c = b[i]
    if 0xC2 <= c <= 0xDF:
        n, cp = 2, c & 0x1F
    elif 0xE0 <= c <= 0xEF:
        n, cp = 3, c & 0x0F
    elif 0xF0 <= c <= 0xF4:
        n, cp = 4, c & 0x07
    else:
        return None, 1
    if i + n > len(b):
        return None, 1
    for k in range(1, n):
        if b[i + k] & 0xC0 != 0x80:
            return None, 1
        cp = (cp << 6) | (b[i + k] & 0x3F)
    c1 = b[i + 1]
    if (c == 0xE0 and c1 < 0xA0) or (c == 0xED and c1 > 0x9F) or (c == 0xF0 and c1 < 0x90) or (c == 0xF4 and c1 > 0x8F):
        return None, 1
    return cp, n


def go_string(s: bytes) -> bytes:
    out = bytearray(b'"')
    i = 0
    while i < len(s):
        c = s[i]
        if c < 0x80:
            if c >= 0x20 and c not in b'"\\<>&':
                out.append(c)
            elif c in b'"\\':
                out += b"\\" + bytes([c])
            elif c == 0x0A:
                out += b"\\n"
            elif c == 0x0D:
                out += b"\\r"
            elif c == 0x09:
                out += b"\\t"
            else:
                out += b"\\u00" + _HEX[c >> 4].encode() + _HEX[c & 15].encode()
            i += 1
            continue
        cp, n = _utf8_decode_rune(s, i)
        if cp is None:
            out += b"\\ufffd"
            i += 1
            continue
        if cp in (0x2028, 0x2029):
            out += b"\\u2028" if cp == 0x2028 else b"\\u2029"
        else:
            out += s[i:i + n]
        i += n
    out += b'"'
    return bytes(out)


def _b(x) -> bytes:
    return x if isinstance(x, bytes) else x.encode("utf-8", "surrogatepass")


def marshal_value(v: Dict) -> bytes:
    items = sorted((_b(k), _b(x)) for k, x in v.items())
    return b"{" + b",".join(go_string(k) + b":" + go_string(x) for k, x in items) + b"}"


def marshal_diff(diff: Dict[int, Dict]) -> bytes:
    items = sorted((str(int(ts)).encode(), v) for ts, v in diff.items())
    return b"{" + b",".join(go_string(k) + b":" + marshal_value(v) for k, v in items) + b"}"


def go_atoi(s: str):
    """strconv.Atoi on a 64-bit platform; None on error."""
    if not s:
        return None
    i, neg = 0, False
    if s[0] in "+-":
        neg, i = s[0] == "-", 1
        if len(s) == 1:
            return None
    if not all("0" <= ch <= "9" for ch in s[i:]):
        return None
    v = int(s[i:]) * (-1 if neg else 1)
    return v if -(2**63) <= v < 2**63 else None


def _fix_surrogates(s: str) -> str:
    # Go replaces unpaired surrogate escapes with U+FFFD
    return "".join("\ufffd" if 0xD800 <= ord(ch) <= 0xDFFF else ch for ch in s)


class _Obj(list):
    """A JSON object as its (key, value) pairs, duplicates kept."""


def ingest(data: bytes) -> Tuple[int, Dict[int, Dict[str, str]]]:
    def bad_const(x):
        raise ValueError(x)

    try:                                   # pairs kept as lists: every duplicate is type-checked
        top = json.loads(data.decode("utf-8"), object_pairs_hook=_Obj, parse_constant=bad_const)
    except ValueError:
        return 1, {}
    if top is None:
        return 0, {}
    if not isinstance(top, _Obj):
        return 1, {}
    for _, v in top:                       # a type error anywhere fails Unmarshal, even if overwritten later
        if v is None:
            continue
        if not isinstance(v, _Obj) or not all(isinstance(x, str) or x is None for _, x in v):
            return 1, {}
    m: Dict[str, Dict[str, str]] = {}
    for k, v in top:                       # duplicate keys: the last wins (both levels)
        m[_fix_surrogates(k)] = {_fix_surrogates(kk): _fix_surrogates(vv) if vv is not None else ""
                                 for kk, vv in (v or [])}
    order = sorted(m, key=lambda x: x.encode("utf-8", "surrogatepass"))
    ts = {}
    for k in order:
        a = go_atoi(k)
        if a is None:
            return 2, {}
        ts[k] = a
    remote: Dict[int, Dict[str, str]] = {}
    for k in order:
        remote[ts[k]] = m[k]
    return 0, remote
