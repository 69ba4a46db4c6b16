"""GPU: the segmented primitives under the gossip assembly (crdt_amd.gossip,
csrc/gossip.hip, csrc/scan.hpp) against numpy: the single-pass scan
(crdt_counts_to_offsets, crdt_seg_offsets), the two-array segmented copy with
a per-segment delta (crdt_seg_copy2, thread and workgroup forms) and the
fused offsets + gather (crdt_seg_gather2).  Sizes straddle the 2048-item scan
tile; segments are empty, single, long and mixed; codes mix both sources."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _p(t):
    return None if t is None else t.data_ptr()


def _dev(a, eng):
    return torch.from_numpy(np.ascontiguousarray(a)).to(eng.device)


def _case(rng, n_seg, max_len, na_seg=300, nb_seg=200):
    la = rng.integers(0, max_len + 1, na_seg)
    lb = rng.integers(0, max_len + 1, nb_seg)
    a_off = np.concatenate([[0], np.cumsum(la)]).astype(np.int64)
    b_off = np.concatenate([[0], np.cumsum(lb)]).astype(np.int64)
    code = np.where(rng.random(n_seg) < 0.5, rng.integers(0, na_seg, n_seg), -(rng.integers(0, nb_seg, n_seg) + 1))
    return code.astype(np.int64), a_off, b_off


def _np_layout(code, a_off, b_off, base):
    lens = np.where(code >= 0, a_off[np.maximum(code, 0) + 1] - a_off[np.maximum(code, 0)],
                    b_off[np.maximum(-code - 1, 0) + 1] - b_off[np.maximum(-code - 1, 0)])
    return np.concatenate([[0], np.cumsum(lens)]).astype(np.int64) + base


def _np_copy(code, a_off, b_off, a, b, delta=None):
    parts = []
    for s, c in enumerate(code):
        src, off, k = (a, a_off, c) if c >= 0 else (b, b_off, -c - 1)
        x = src[off[k]:off[k + 1]].copy()
        if delta is not None:
            x = x + delta[s]
        parts.append(x)
    return np.concatenate(parts) if parts else np.zeros(0, a.dtype)


@pytest.mark.parametrize("n", [0, 1, 2047, 2048, 2049, 300_001])
def test_counts_to_offsets(eng, n):
    rng = np.random.default_rng(n)
    c = rng.integers(0, 1 << 20, n).astype(np.uint32)
    c[: n // 7] = 0xFFFFFFFF                                    # large counts: the 64-bit sums
    out = torch.empty(n + 1, dtype=torch.int64, device=eng.device)
    eng._call("crdt_counts_to_offsets", _p(_dev(c.view(np.int32), eng)) if n else None, n, 12345, _p(out))
    exp = np.concatenate([[0], np.cumsum(c.astype(np.uint64))]).astype(np.uint64) + np.uint64(12345)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64), exp)
    assert eng.device_status() == 0


@pytest.mark.parametrize("n_seg,max_len", [(1, 0), (5, 3), (2048, 2), (2049, 1), (70_000, 3), (9, 5000)])
def test_seg_offsets_and_gather2(eng, n_seg, max_len):
    rng = np.random.default_rng(n_seg * 31 + max_len)
    code, a_off, b_off = _case(rng, n_seg, max_len)
    a0 = rng.integers(0, 1 << 31, max(a_off[-1], 1)).astype(np.int32)
    a1 = rng.integers(0, 1 << 31, max(a_off[-1], 1)).astype(np.int32)
    b0 = rng.integers(0, 1 << 31, max(b_off[-1], 1)).astype(np.int32)
    b1 = rng.integers(0, 1 << 31, max(b_off[-1], 1)).astype(np.int32)
    base = 77
    exp_off = _np_layout(code, a_off, b_off, base)
    dc, da, db = _dev(code, eng), _dev(a_off, eng), _dev(b_off, eng)
    off = torch.empty(n_seg + 1, dtype=torch.int64, device=eng.device)
    eng._call("crdt_seg_offsets", n_seg, _p(dc), _p(da), _p(db), base, _p(off))
    np.testing.assert_array_equal(off.cpu().numpy(), exp_off)

    total = int(exp_off[-1] - base)
    d0 = torch.full((base + total + 1,), -1, dtype=torch.int32, device=eng.device)
    d1 = torch.full_like(d0, -1)
    off2 = torch.empty_like(off)
    t = [_dev(x, eng) for x in (a0, b0, a1, b1)]
    eng._call("crdt_seg_gather2", n_seg, _p(dc), _p(da), _p(db), base, _p(off2), 4, _p(t[0]), _p(t[1]), _p(d0),
              _p(t[2]), _p(t[3]), _p(d1))
    np.testing.assert_array_equal(off2.cpu().numpy(), exp_off)
    g0, g1 = d0.cpu().numpy(), d1.cpu().numpy()
    np.testing.assert_array_equal(g0[base:base + total], _np_copy(code, a_off, b_off, a0, b0))
    np.testing.assert_array_equal(g1[base:base + total], _np_copy(code, a_off, b_off, a1, b1))
    assert (g0[:base] == -1).all() and g0[base + total] == -1       # nothing written outside the layout
    assert eng.device_status() == 0


@pytest.mark.parametrize("wide", [0, 1])
@pytest.mark.parametrize("n_seg,max_len", [(3, 20_000), (700, 40), (40_000, 2)])
def test_seg_copy2_delta(eng, wide, n_seg, max_len):
    rng = np.random.default_rng(n_seg + wide)
    code, a_off, b_off = _case(rng, n_seg, max_len, na_seg=50, nb_seg=40)
    a0 = rng.integers(-(1 << 62), 1 << 62, a_off[-1]).astype(np.int64)
    b0 = rng.integers(-(1 << 62), 1 << 62, max(b_off[-1], 1)).astype(np.int64)
    a1 = rng.integers(0, 1 << 40, a_off[-1]).astype(np.int64)
    b1 = rng.integers(0, 1 << 40, max(b_off[-1], 1)).astype(np.int64)
    delta = rng.integers(-(1 << 62), 1 << 62, n_seg).astype(np.int64)
    off = _np_layout(code, a_off, b_off, 0)
    total = int(off[-1])
    d0 = torch.empty(max(total, 1), dtype=torch.int64, device=eng.device)
    d1 = torch.empty_like(d0)
    t = [_dev(x, eng) for x in (code, a_off, b_off, off, a0, b0, delta, a1, b1)]
    eng._call("crdt_seg_copy2", n_seg, *[_p(x) for x in t[:4]], 8, _p(t[4]), _p(t[5]), _p(d0), _p(t[6]), _p(t[7]),
              _p(t[8]), _p(d1), wide)
    with np.errstate(over="ignore"):
        exp0 = _np_copy(code, a_off, b_off, a0.view(np.uint64), b0.view(np.uint64), delta.view(np.uint64))
    np.testing.assert_array_equal(d0.cpu().numpy()[:total].view(np.uint64), exp0)
    np.testing.assert_array_equal(d1.cpu().numpy()[:total], _np_copy(code, a_off, b_off, a1, b1))
