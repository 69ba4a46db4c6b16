"""CPU: the cgo binding (go/crdt/*.go, uncompiled here: no Go toolchain)
matches include/crdt_amd.h symbol for symbol -- every C.crdt_* function it
calls is declared and gets as many arguments as its prototype takes, every
C.CRDT_* constant and C.crdt_* type it names exists (VERDICT r05 item 8;
reference: main.go:23-33, :35, :102)."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO_FILES = sorted(glob.glob(os.path.join(ROOT, "go", "crdt", "*.go")))


def _header():
    with open(os.path.join(ROOT, "include", "crdt_amd.h")) as f:
        return re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)


def _split_args(s):
    """Top-level comma split of a call's argument text."""
    depth, cur, out = 0, "", []
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return out


def _calls(src, prefix):
    """(name, argument count) of every C.<prefix>...( call in Go source."""
    out = []
    for m in re.finditer(r"\bC\.(" + prefix + r"\w*)\(", src):
        i, depth = m.end(), 1
        while depth:
            depth += {"(": 1, ")": -1}.get(src[i], 0)
            i += 1
        out.append((m.group(1), len(_split_args(src[m.end():i - 1]))))
    return out


def _prototypes():
    protos = {}
    for m in re.finditer(r"^\s*(?:const\s+)?\w+\s*\*?\s*(crdt_\w+)\s*\(([^;]*?)\)\s*;", _header(), flags=re.M | re.S):
        args = m.group(2).strip()
        protos[m.group(1)] = 0 if args in ("", "void") else len(_split_args(args))
    return protos


def test_go_files_exist_with_build_tags():
    names = {os.path.basename(p) for p in GO_FILES}
    assert {"crdt_gpu.go", "population_gpu.go"} <= names
    assert os.path.exists(os.path.join(ROOT, "go", "crdt", "go.mod"))
    for p in GO_FILES:
        with open(p) as f:
            assert f.readline().strip() == "//go:build cgo && rocm", p


def test_reference_shaped_server_surface():
    with open(os.path.join(ROOT, "go", "crdt", "crdt_gpu.go")) as f:
        src = f.read()
    assert "func NewServer(port int, initialState Data, friendList []string) *Server" in src   # main.go:102
    assert "func (server *Server) merge()" in src                                             # main.go:35
    for name, typ in (("InitialState", "Data"), ("CurrentState", "Data"), ("Diff", r"\*gpuLog"),
                      ("RemoteDiff", r"\*gpuLog"), ("Port", "int"), ("LastReceived", "int64"),
                      ("FriendList", r"\[\]string"), ("Alive", "bool"), ("Lock", r"sync\.Mutex")):  # main.go:23-33
        assert re.search(r"^\t" + name + r"\s+" + typ + r"$", src, flags=re.M), name


def test_every_c_call_matches_the_header():
    protos = _prototypes()
    seen = set()
    for p in GO_FILES:
        with open(p) as f:
            src = f.read()
        for name, nargs in _calls(src, "crdt_"):
            assert name in protos, f"{os.path.basename(p)}: C.{name} is not declared in crdt_amd.h"
            assert nargs == protos[name], f"{os.path.basename(p)}: C.{name} called with {nargs} args, " \
                                          f"header takes {protos[name]}"
            seen.add(name)
    assert {"crdt_server_merge", "crdt_server_new", "crdt_servers_merge", "crdt_shard_fold_max_u64",
            "crdt_population_round_wire"} <= seen


def test_every_c_constant_and_type_is_declared():
    hdr = _header()
    for p in GO_FILES:
        with open(p) as f:
            src = f.read()
        for const in set(re.findall(r"\bC\.(CRDT_\w+)", src)):
            assert re.search(r"\b" + const + r"\b", hdr), const
        for typ in set(re.findall(r"\bC\.(crdt_\w+)\b(?!\()", src)):
            assert re.search(r"\b(typedef\s+struct\s+" + typ + r"\b|}\s*" + typ + r"\s*;|typedef[^;]*\b" + typ + r"\s*;)",
                             hdr), typ
