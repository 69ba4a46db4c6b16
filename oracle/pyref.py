"""Pure-Python literal restatement of (*Server).merge() -- small cases only.

TEST INFRASTRUCTURE ONLY.  A line-by-line transliteration of
/root/reference/main.go:35-100 over Python dicts, used to cross-check the C
restatement (oracle/crdt_oracle.c) and the packers on the KAT fixtures.

Model of the reference's dynamic types:
  * a Diff value that is a :class:`Command` instance is a local write
    (`*Command`, main.go:187); anything else is a remote `map[string]string`
    (main.go:245-255, inserted unchanged by main.go:67-68).
"""
from __future__ import annotations


class Command(dict):
    """`type Command map[string]string` (main.go:21), stored by pointer."""


def go_atoi(s: str):
    """strconv.Atoi (Go 1.18, 64-bit int): (ok, value)."""
    if not s:
        return False, 0
    i, neg = 0, False
    if s[0] in "+-":
        neg, i = s[0] == "-", 1
        if len(s) == 1:
            return False, 0
    acc = 0
    for ch in s[i:]:
        if not ("0" <= ch <= "9"):
            return False, 0
        acc = acc * 10 + (ord(ch) - 48)
        if acc > 2**64 - 1:
            return False, 0
    if not neg and acc >= 2**63:
        return False, 0
    if neg and acc > 2**63:
        return False, 0
    return True, -acc if neg else acc


def _wrap64(x: int) -> int:
    x &= 2**64 - 1
    return x - 2**64 if x >= 2**63 else x


def merge(diff: dict, remote: dict):
    """Returns (new_diff, current_state); inputs are not modified."""
    diff = dict(diff)
    has_ids = sorted(diff)                 # Diff.Keys(), ascending (main.go:45)
    out_ids = sorted(remote)               # RemoteDiff.Keys() (main.go:47)
    i = j = 0
    while i < len(has_ids) and j < len(out_ids):            # main.go:49
        cd, cr = has_ids[i], out_ids[j]                      # main.go:52-53
        if cd == cr:                                         # main.go:54-65: local kept
            i += 1
            j += 1
        elif cd > cr:                                        # main.go:66-69
            diff[cr] = remote[cr]
            j += 1
        else:                                                # main.go:70-72
            i += 1
    state: dict = {}                                         # main.go:76
    for ts in sorted(diff, reverse=True):                    # main.go:77-78 (End/Prev)
        value = diff[ts]
        if type(value).__name__ == "Command":                # *Command fails the assertion (:80)
            continue
        for key, valx in value.items():                      # main.go:81
            if key not in state:                             # main.go:82-86
                state[key] = valx
                continue
            ok, curr = go_atoi(state[key])                   # main.go:87-90
            if not ok:
                continue
            ok, change = go_atoi(valx)                       # main.go:91-94
            if not ok:
                continue
            state[key] = str(_wrap64(curr + change))         # main.go:95-96 (Itoa)
    return diff, state


def add_command(diff: dict, state: dict, ts: int, data: dict, alive: bool = True) -> int:
    """AddCommand (main.go:173-215) after the request body's JSON decode:
    Diff.Put(ts, &data) (main.go:187; a same-ms write replaces the entry),
    then the local apply to CurrentState (main.go:188-207), keys in sorted
    order (Go's map order is random: sorted order is one legal execution).
    Mutates diff and state; returns the HTTP status (200 / 500 / 502)."""
    if not alive:                                            # main.go:209-212
        return 502
    diff[ts] = Command(data)                                 # main.go:187
    for key in sorted(data):                                 # main.go:188
        value = data[key]
        if key not in state:                                 # main.go:189-193: insert, RETURN
            state[key] = value
            return 200
        ok, curr = go_atoi(state[key])                       # main.go:195-199
        if not ok:
            return 500
        ok, change = go_atoi(value)                          # main.go:200-204
        if not ok:
            return 500
        state[key] = str(_wrap64(curr + change))             # main.go:205-206 (Itoa)
    return 200                                               # main.go:207-208
