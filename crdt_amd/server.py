"""Reference-shaped `Server` over the C++ host mirror (csrc/server.hip).

Mirrors the Go API of /root/reference/main.go so callers read like the
reference:

    s = NewServer(8080, {}, friends)          # main.go:102-113
    s.Diff.Put(ts, Command({"a": "1"}))       # local write  (main.go:187)
    s.RemoteDiff.Put(ts, {"a": "3"})          # gossip ingest (main.go:255)
    s.merge()                                 # main.go:35-100, on the GPU
    s.CurrentState                            # map[string]string

The merge runs in libcrdt_amd.so's batched RefMerge kernels; `merge_servers`
merges many servers in one device call.  No CPU path exists.
"""
from __future__ import annotations

import ctypes as C
from typing import Tuple, Dict, Iterable, List, Sequence

from . import _lib
from ._lib import call
from .refmerge import Command, Data  # noqa: F401  (re-exported: main.go:19-21)


def Int64Comparator(a: int, b: int) -> int:
    """utils.Int64Comparator (main.go:106-107), via the C-ABI."""
    return _lib.lib().crdt_compare_int64(a, b)


def _enc(x) -> bytes:
    return x if isinstance(x, bytes) else x.encode("utf-8", "surrogatepass")


def _dec(b: bytes) -> str:
    # Go strings are byte strings: bytes that are not UTF-8 survive as lone
    # surrogates (surrogateescape) so a Get round-trips what a Put stored.
    return b.decode("utf-8", "surrogateescape")


def _kv_arrays(d: Dict[str, str]):
    items = [(_enc(k), _enc(v)) for k, v in d.items()]
    n = len(items)
    keys = (C.c_char_p * max(n, 1))(*[k for k, _ in items])
    vals = (C.c_char_p * max(n, 1))(*[v for _, v in items])
    kl = (C.c_size_t * max(n, 1))(*[len(k) for k, _ in items])
    vl = (C.c_size_t * max(n, 1))(*[len(v) for _, v in items])
    return keys, kl, vals, vl, n


class _TreeMap:
    """The Put side of a gods treemap (main.go:26-27) bound to one server."""

    def __init__(self, srv: "Server", remote: bool):
        self._srv, self._remote = srv, remote

    def Put(self, ts: int, value: Dict[str, str]) -> None:
        keys, kl, vals, vl, n = _kv_arrays(value)
        if self._remote:
            call("crdt_server_remote_put", self._srv._h, int(ts), keys, kl, vals, vl, n)
        else:
            local = 1 if isinstance(value, Command) else 0
            call("crdt_server_diff_put", self._srv._h, int(ts), local, keys, kl, vals, vl, n)

    def Keys(self) -> List[int]:
        return [t for t, _ in self._srv._diff_entries()] if not self._remote else self._remote_keys()

    def _remote_keys(self) -> List[int]:
        n = C.c_size_t()
        call("crdt_server_remote_keys", self._srv._h, None, 0, C.byref(n))
        cap = n.value
        ts = (C.c_int64 * max(cap, 1))()
        call("crdt_server_remote_keys", self._srv._h, ts, cap, C.byref(n))
        return [ts[i] for i in range(min(cap, n.value))]

    def Get(self, ts: int) -> Tuple[Dict[str, str] | None, bool]:
        """treemap Get (gods v1.18.1): (value, found); the value as a dict."""
        k, kl, v, vl, n = C.c_void_p(), C.c_size_t(), C.c_void_p(), C.c_size_t(), C.c_size_t()
        h, r = self._srv._h, 1 if self._remote else 0
        rc = _lib.lib().crdt_server_entry_at(h, r, int(ts), 0, C.byref(k), C.byref(kl), C.byref(v), C.byref(vl),
                                             C.byref(n))
        if rc == -6:                       # CRDT_E_RANGE: absent
            return None, False
        if rc < 0:
            _lib.check("crdt_server_entry_at", rc)
        out = {}
        for i in range(n.value):
            call("crdt_server_entry_at", h, r, int(ts), i, C.byref(k), C.byref(kl), C.byref(v), C.byref(vl),
                 C.byref(n))
            out[_dec(C.string_at(k.value, kl.value) if kl.value else b"")] = \
                _dec(C.string_at(v.value, vl.value) if vl.value else b"")
        return out, True

    def Size(self) -> int:
        n = C.c_size_t()
        call("crdt_server_remote_len" if self._remote else "crdt_server_diff_len", self._srv._h, C.byref(n))
        return n.value


class Server:
    """Host handle of one replica (main.go:23-33)."""

    def __init__(self, eng, port: int, initial_state: Dict[str, str] | None = None,
                 friend_list: Sequence[str] = ()):
        self._eng = eng                       # None: host-only (codec, AddCommand; no merge)
        h = C.c_void_p()
        call("crdt_server_new", eng.ctx if eng is not None else None, int(port), C.byref(h))
        self._h = h
        if eng is not None:
            eng._depend(self)                 # freed before the context its device Diff lives on
        self.Port = port
        self.InitialState = dict(initial_state or {})
        self.FriendList = list(friend_list)
        self.LastReceived = 0
        self.Diff = _TreeMap(self, remote=False)
        self.RemoteDiff = _TreeMap(self, remote=True)
        if self.InitialState:
            keys, kl, vals, vl, n = _kv_arrays(self.InitialState)
            call("crdt_server_init_state", h, keys, kl, vals, vl, n)

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.lib().crdt_server_free(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def merge(self) -> None:
        """(*Server).merge() -- main.go:35-100, bit-exact, on the GPU."""
        if self._eng is None:
            raise _lib.CrdtLibraryError("host-only Server (no engine): merge() runs on the GPU")
        self._eng._bind()
        call("crdt_server_merge", self._h)

    def Gossip(self) -> Tuple[int, bytes]:
        """GET /gossip (main.go:153-170): (HTTP status, body) -- 200 with
        Diff.ToJSON() (main.go:159) or 502 "Unreachable"."""
        n, st = C.c_size_t(), C.c_int()
        while True:
            buf = C.create_string_buffer(max(n.value, 1))
            rc = _lib.lib().crdt_server_gossip_json(self._h, buf, n.value, C.byref(n), C.byref(st))
            if rc != -6:                        # CRDT_E_RANGE: *n = size needed; retry (Diff may grow)
                break
        if rc < 0:
            _lib.check("crdt_server_gossip_json", rc)
        return st.value, buf.raw[: n.value]

    def GossipBinary(self) -> Tuple[int, bytes]:
        """The binary SoA form of the Gossip response (crdt_server_gossip_binary)."""
        n, st = C.c_size_t(), C.c_int()
        while True:
            buf = C.create_string_buffer(max(n.value, 1))
            rc = _lib.lib().crdt_server_gossip_binary(self._h, buf, n.value, C.byref(n), C.byref(st))
            if rc != -6:
                break
        if rc < 0:
            _lib.check("crdt_server_gossip_binary", rc)
        return st.value, buf.raw[: n.value]

    def IngestBinary(self, data: bytes) -> int:
        """Binary SoA pull decode: 0 = ingested into RemoteDiff, 1 = malformed."""
        out = C.c_int()
        call("crdt_server_ingest_binary", self._h, bytes(data), len(data), C.byref(out))
        return out.value

    def SetAlive(self, alive: bool) -> None:
        """AliveState handler (main.go:141-151) after ParseBool."""
        call("crdt_server_set_alive", self._h, 1 if alive else 0)

    def IngestGossip(self, data: bytes) -> int:
        """The gossip pull's decode (main.go:245-256).  Returns 0 = ingested
        into RemoteDiff (merge() next, main.go:257), 1 = bad JSON / shape, round
        skipped (main.go:247-249), 2 = a key failed Atoi, the reference's gossip
        goroutine returns (main.go:252-253)."""
        out = C.c_int()
        call("crdt_server_ingest_json", self._h, bytes(data), len(data), C.byref(out))
        return out.value

    def AddCommand(self, ts_ms: int, data: Dict[str, str]) -> int:
        """POST /data after decoding (main.go:173-215); returns the HTTP status."""
        keys, kl, vals, vl, n = _kv_arrays(data)
        st = C.c_int()
        call("crdt_server_add_command", self._h, int(ts_ms), keys, kl, vals, vl, n, C.byref(st))
        return st.value

    def _diff_entries(self):
        n = C.c_size_t()
        call("crdt_server_diff_keys", self._h, None, None, 0, C.byref(n))
        cap = n.value
        ts = (C.c_int64 * max(cap, 1))()
        loc = (C.c_uint8 * max(cap, 1))()
        call("crdt_server_diff_keys", self._h, ts, loc, cap, C.byref(n))
        return [(ts[i], "local" if loc[i] else "remote") for i in range(min(cap, n.value))]

    @property
    def DiffSignature(self) -> List[list]:
        """[[ts, "local"|"remote"], ...] ascending (Diff.Keys(), main.go:45)."""
        return [[t, o] for t, o in self._diff_entries()]

    @property
    def CurrentState(self) -> Dict[str, str]:
        n = C.c_size_t()
        call("crdt_server_state_len", self._h, C.byref(n))
        out = {}
        k, kl, v, vl = C.c_void_p(), C.c_size_t(), C.c_void_p(), C.c_size_t()
        for i in range(n.value):
            call("crdt_server_state_at", self._h, i, C.byref(k), C.byref(kl), C.byref(v), C.byref(vl))
            key = C.string_at(k.value, kl.value) if kl.value else b""
            val = C.string_at(v.value, vl.value) if vl.value else b""
            out[key.decode("utf-8", "surrogatepass")] = val.decode("utf-8", "surrogatepass")
        return out


def NewServer(port: int, initialState: Dict[str, str], friendList: Sequence[str], eng=None) -> Server:
    """NewServer (main.go:102-113)."""
    if eng is None:
        from .engine import Engine
        eng = Engine(0)
    return Server(eng, port, initialState, friendList)


def merge_servers(servers: Iterable[Server]) -> None:
    """merge() of every server in ONE batched device call (same GPU)."""
    servers = list(servers)
    if not servers:
        return
    servers[0]._eng._bind()
    arr = (C.c_void_p * len(servers))(*[s._h.value for s in servers])
    call("crdt_servers_merge", arr, len(servers))
