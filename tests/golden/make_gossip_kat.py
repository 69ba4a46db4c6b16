#!/usr/bin/env python3
"""Writes tests/golden/gossip_json_kat.json: known answers for the gossip
wire format (main.go:153-170 serve, :245-256 pull), WRITTEN BY HAND from the
reference's source and Go 1.18 encoding/json's documented behaviour -- not
computed by any code under test.  Byte strings are stored as latin-1
(one char per byte) so invalid UTF-8 survives the JSON file."""
import json
import os

L = lambda b: b.decode("latin-1")

MARSHAL = [
    # Diff {ts: (local?, {k: v})} -> response body
    {"name": "byte-string key order, local and remote values, empty map",
     "diff": [[10, True, {"z": "1"}], [2, False, {"b": "x", "a": "y"}], [-5, False, {}]],
     "body": '{"-5":{},"10":{"z":"1"},"2":{"a":"y","b":"x"}}'},
    {"name": "numeric vs byte order of keys",
     "diff": [[9, False, {}], [10, False, {}], [-1, False, {}], [100, False, {}]],
     "body": '{"-1":{},"10":{},"100":{},"9":{}}'},
    {"name": "HTML-safe and control escapes",
     "diff": [[1, False, {"k": L(b'<a&b>"q\\\n\r\t\x01\x08\x0c\x1f\x7f')}]],
     "body": '{"1":{"k":"\\u003ca\\u0026b\\u003e\\"q\\\\\\n\\r\\t\\u0001\\u0008\\u000c\\u001f' + '\x7f' + '"}}'},
    {"name": "UTF-8 kept, U+2028/9 escaped, invalid bytes replaced one by one",
     "diff": [[1, False, {"e": L("é".encode()), "l": L("\u2028\u2029".encode()),
                           "x": L(b"\xff"), "t": L(b"\xe2\x82"), "o": L(b"\xc0\x80"), "s": L(b"\xed\xa0\x80")}]],
     "body": '{"1":{"e":"' + L("é".encode()) + '","l":"\\u2028\\u2029","o":"\\ufffd\\ufffd",'
             '"s":"\\ufffd\\ufffd\\ufffd","t":"\\ufffd\\ufffd","x":"\\ufffd"}}'},
    {"name": "int64 extremes as keys",
     "diff": [[-9223372036854775808, False, {}], [9223372036854775807, False, {"a": ""}]],
     "body": '{"-9223372036854775808":{},"9223372036854775807":{"a":""}}'},
]

INGEST = [
    # body -> (outcome, RemoteDiff after)
    {"name": "two entries", "body": '{"5":{"a":"1"},"7":{"b":"2"}}', "outcome": 0,
     "remote": [[5, {"a": "1"}], [7, {"b": "2"}]]},
    {"name": "number member: type error, round skipped", "body": '{"5":{"a":1}}', "outcome": 1, "remote": []},
    {"name": "non-numeric key: goroutine returns", "body": '{"x":{"a":"1"}}', "outcome": 2, "remote": []},
    {"name": "key out of int64 range", "body": '{"9223372036854775808":{}}', "outcome": 2, "remote": []},
    {"name": "not JSON", "body": "not json", "outcome": 1, "remote": []},
    {"name": "null body: nil map, nothing to put", "body": "null", "outcome": 0, "remote": []},
    {"name": "empty object", "body": "{}", "outcome": 0, "remote": []},
    {"name": "duplicate key: the last wins", "body": '{"5":{"a":"1"},"5":{"a":"2"}}', "outcome": 0,
     "remote": [[5, {"a": "2"}]]},
    {"name": "\"01\" and \"1\" both Atoi to 1: byte order, last wins", "body": '{"1":{"a":"2"},"01":{"a":"1"}}',
     "outcome": 0, "remote": [[1, {"a": "2"}]]},
    {"name": "escaped key and values, surrogate pair", "body": '{"\\u0035":{"\\u00e9":"\\ud83d\\ude00"}}',
     "outcome": 0, "remote": [[5, {L("é".encode()): L("\U0001F600".encode())}]]},
    {"name": "lone surrogate -> U+FFFD", "body": '{"5":{"a":"\\ud800x"}}', "outcome": 0,
     "remote": [[5, {"a": L("\ufffdx".encode())}]]},
    {"name": "raw invalid byte -> U+FFFD", "body": L(b'{"5":{"a":"\xff"}}'), "outcome": 0,
     "remote": [[5, {"a": L("\ufffd".encode())}]]},
    {"name": "null value: empty map", "body": '{"5":null}', "outcome": 0, "remote": [[5, {}]]},
    {"name": "null member: zero-value string", "body": '{"5":{"a":null}}', "outcome": 0, "remote": [[5, {"a": ""}]]},
    {"name": "trailing data", "body": "{} x", "outcome": 1, "remote": []},
    {"name": "whitespace everywhere", "body": ' \n{ "5" :\t{ "a" : "1" } } ', "outcome": 0,
     "remote": [[5, {"a": "1"}]]},
    {"name": "plus-signed key", "body": '{"+5":{}}', "outcome": 0, "remote": [[5, {}]]},
    {"name": "raw control character in a string is invalid JSON", "body": '{"5":{"a":"\x01"}}', "outcome": 1,
     "remote": []},
    {"name": "array at the top level", "body": "[]", "outcome": 1, "remote": []},
]

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gossip_json_kat.json")
    with open(out, "w") as f:
        json.dump({"marshal": MARSHAL, "ingest": INGEST}, f, indent=1)
    print(out)
