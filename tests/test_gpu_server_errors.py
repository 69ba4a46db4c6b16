"""GPU: error paths at the C-ABI.

* A failed device merge through crdt_server_merge (fault injection
  "fail.refmerge": the RefMerge call fails before touching the device)
  returns its status and leaves Diff, RemoteDiff and CurrentState exactly as
  they were, the server Alive again (its lock released) -- and the next
  merge() succeeds with the KAT answer.
* CRDT_E_RANGE where the replay's packing would overflow: a batch whose
  merge sequences could exceed 2^32 entries (best = rank << 32 | string id)
  and a shard index past the shard << 40 packing.
* A remote entry pulled as JSON null is a nil map: after merge() inserts it,
  the Gossip handler re-serves it as `null` (json.Marshal of a nil
  map[string]string, main.go:159), over the JSON and the binary codec.
"""
import ctypes as C

import pytest
from knobs import set_knob
import torch

from crdt_amd import _lib
from crdt_amd.server import Server
from refmerge_util import kat_inputs, load_kats

pytestmark = pytest.mark.gpu


def _server_from(eng, diff, remote, port=8080):
    s = Server(eng, port)
    for ts, v in diff.items():
        s.Diff.Put(ts, v)
    for ts, v in remote.items():
        s.RemoteDiff.Put(ts, v)
    return s


@pytest.mark.diag
def test_failed_merge_leaves_server_untouched(eng):
    kat = next(k for k in load_kats() if k["name"].startswith("KAT-1"))
    diff, remote = kat_inputs(kat)
    s = _server_from(eng, diff, remote)
    before = (s.DiffSignature, s.RemoteDiff.Keys(), s.CurrentState, [s.RemoteDiff.Get(t) for t in remote])
    set_knob(b"fail.refmerge", 1)
    with pytest.raises(_lib.CrdtError) as ei:
        s.merge()
    assert ei.value.status == -3                                   # CRDT_E_NOMEM, as injected
    after = (s.DiffSignature, s.RemoteDiff.Keys(), s.CurrentState, [s.RemoteDiff.Get(t) for t in remote])
    assert after == before
    assert s.Gossip()[0] == 200                                    # Alive again, lock released
    s.merge()                                                      # the failpoint is spent
    assert s.DiffSignature == kat["diff"] and s.CurrentState == kat["state"]
    s.close()


def test_refmerge_range_guards(eng):
    t = torch.zeros(16, dtype=torch.int64, device=eng.device)
    p = t.data_ptr()
    cin = _lib.crdt_refmerge_in(1, 4, 2**32 - 1, 1, 1, 1, p, p, p, p, p, p, p, p, p, p, p)
    cout = _lib.crdt_refmerge_out(p, p, p, p, p, p, p)
    rc = _lib.lib().crdt_refmerge_batch(eng.ctx, C.byref(cin), C.byref(cout))
    assert rc == -6                                               # CRDT_E_RANGE before any launch
    acc = _lib.crdt_refmerge_acc(p, p, p)
    assert _lib.lib().crdt_refmerge_acc_rank(eng.ctx, C.byref(acc), 4, 1 << 23, p) == -6
    assert _lib.lib().crdt_refmerge_acc_rank(eng.ctx, C.byref(acc), 4, (1 << 23) - 1, p) == 0
    eng.sync()


def test_null_ingest_is_reserved_as_null(eng):
    from crdt_amd.refmerge import Command
    s = Server(eng, 8081)
    s.Diff.Put(100, Command({"z": "0"}))
    assert s.IngestGossip(b'{"5":null,"6":{"a":"1"},"7":{"a":"2"}}') == 0
    s.merge()
    assert s.CurrentState == {"a": "3"}
    st, body = s.Gossip()
    assert st == 200 and body == b'{"100":{"z":"0"},"5":null,"6":{"a":"1"},"7":{"a":"2"}}'
    # the binary codec carries the nil flag too
    b = Server(eng, 8082)
    b.Diff.Put(1000, Command({"q": "1"}))
    assert b.IngestBinary(s.GossipBinary()[1]) == 0
    b.merge()
    assert b.Gossip()[1] == b'{"100":{"z":"0"},"1000":{"q":"1"},"5":null,"6":{"a":"1"},"7":{"a":"2"}}'
    s.close()
    b.close()


@pytest.mark.diag
def test_inconsistent_bitmaps_fail_merge_cleanly(eng):
    """fail.zero_bits: the RefMerge bitmaps zeroed between its count and tile
    passes.  The tile pass raises CRDT_DEV_RANGE instead of reading past the
    logs; merge() returns CRDT_E_DEVICE with Diff, RemoteDiff and
    CurrentState untouched and the server Alive -- on the first (host-built)
    merge and on a device-resident one -- and the next merge() is exact."""
    kat = next(k for k in load_kats() if k["name"].startswith("KAT-1"))
    diff, remote = kat_inputs(kat)
    s = _server_from(eng, diff, remote)
    for resident in (False, True):
        before = (s.DiffSignature, s.RemoteDiff.Keys(), s.CurrentState, [s.RemoteDiff.Get(t) for t in remote])
        set_knob(b"fail.zero_bits", 1)
        with pytest.raises(_lib.CrdtError) as ei:
            s.merge()
        assert ei.value.status == -8                               # CRDT_E_DEVICE
        after = (s.DiffSignature, s.RemoteDiff.Keys(), s.CurrentState, [s.RemoteDiff.Get(t) for t in remote])
        assert after == before, f"resident={resident}"
        assert s.Gossip()[0] == 200                                # Alive again, lock released
        s.merge()
        assert s.DiffSignature == kat["diff"] and s.CurrentState == kat["state"]
        for t, v in remote.items():                                # the same pull again (KAT-5: idempotent)
            s.RemoteDiff.Put(t, v)
    assert eng.device_status(clear=True) & 2                       # the raised flags stay for the caller
    s.close()


@pytest.mark.diag
def test_refmerge_batch_inconsistent_bitmaps_flag(eng):
    """The batched call: the flag is raised (crdt_ctx_device_status), no fault."""
    from crdt_amd import refmerge, synth
    h = synth.refmerge_packed(17, 6, 9000)
    d = refmerge.to_device(h, eng.device)
    set_knob(b"fail.zero_bits", 1)
    eng.refmerge_batch(d)
    assert eng.device_status(clear=True) == 2
    eng.refmerge_batch(d)
    assert eng.device_status(clear=True) == 0
