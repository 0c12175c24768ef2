"""GPU parity for the paths round 1 left unchecked: the full-size C5 mixed
batch (Mixed wrapper with full C4-size Big members) against the reference
oracle, concurrent launches on two streams of ONE context (per-stream scratch),
and descriptors created from device memory (the RCCL-broadcast path)."""
import ctypes as C
import random

import numpy as np
import pytest

import oracle
from dynamicgo_amd import _lib, conv, thrift as T, workloads as W

pytestmark = pytest.mark.gpu


def _checker():
    return oracle.RefOracle() or oracle.PortOracle()


class DevBatch:
    """One batch resident on cuda:0 (slots = dg_slot_bound)."""

    def __init__(self, msgs):
        import torch
        dev = torch.device("cuda:0")
        a, off = W.arena(msgs)
        n = len(msgs)
        lens = np.diff(off).astype(np.int64)
        self.slots = np.zeros(n + 1, dtype=np.int64)
        np.cumsum((lens * 4 + 64 + 7) & ~7, out=self.slots[1:])
        self.n = n
        self.max_len = int(lens.max()) if n else 0
        self.json = torch.from_numpy(a).to(dev)
        self.in_off = torch.from_numpy(off.astype(np.int64)).to(dev)
        self.out = torch.zeros(int(self.slots[-1]) + 64, dtype=torch.uint8, device=dev)
        self.out_off = torch.from_numpy(self.slots).to(dev)
        self.out_len = torch.zeros(n, dtype=torch.int32, device=dev)
        self.ret = torch.zeros(n, dtype=torch.int64, device=dev)

    def launch(self, ctx, dh, root, flags, stream):
        _lib.check(_lib.lib().dg_j2t_batch_device(
            ctx.h, dh, root, self.json.data_ptr(), self.in_off.data_ptr(), self.n, flags, self.out.data_ptr(),
            self.out_off.data_ptr(), self.out_len.data_ptr(), self.ret.data_ptr(), None, stream))

    def results(self):
        o, ol, r = self.out.cpu().numpy(), self.out_len.cpu().numpy(), self.ret.cpu().numpy()
        outs = [o[self.slots[i]:self.slots[i] + ol[i]].tobytes() if r[i] == 0 else b"" for i in range(self.n)]
        return [int(x) for x in r], outs


def _oracle_all(fl, msgs, flags=1):
    chk = _checker()
    a, off = W.arena(msgs)
    er, eo = chk.j2t_arena(fl, a, off, flags, nthreads=8)
    return [int(x) for x in er], eo


def test_c5_mixed_full_size_vs_oracle():
    """C5's generator at large_scale=1.0: 2400 Mixed messages (16 full-size
    Big members of ~85 KiB, 238 Nested, the rest Flat) on the hybrid route
    (small kernel + wave kernel + exact list pass), byte-exact vs the oracle."""
    msgs = W.gen_mixed_batch(random.Random(45), 2400)
    assert sum(m.startswith(b'{"Big"') for m in msgs) >= 8
    fl = T.flatten(W.mixed_desc())
    ctx = conv.default_context()
    ctx.stats(reset=True)
    outs, rets = __import__("test_gpu_parity")._raw_batch(fl, msgs, 1)
    bails, deeps = ctx.stats(reset=True)
    er, eo = _oracle_all(fl, msgs)
    assert [int(r) for r in rets] == er
    assert outs == eo
    assert (bails, deeps) == (0, 0)


@pytest.mark.parametrize("cfg", ["c3", "c5"])
def test_two_streams_one_context_vs_oracle(cfg):
    """Chunks of one batch launched alternately on two streams of the SAME
    context with no synchronisation between them: every list, counter and
    workspace is per stream, so every message must still be exact."""
    import torch
    if cfg == "c3":
        td, msgs = W.nesting_i64_desc(), W.gen_nested_batch(random.Random(43), 6000)
    else:
        td, msgs = W.mixed_desc(), W.gen_mixed_batch(random.Random(46), 6000, large_scale=0.25)
    fl = T.flatten(td)
    ctx = conv.Context(0)
    try:
        dh = ctx.desc(fl)
        chunks = [msgs[i:i + 750] for i in range(0, len(msgs), 750)]
        bs = [DevBatch(c) for c in chunks]
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        torch.cuda.synchronize()
        for rep in range(3):  # several rounds: counters must self-reset per stream
            for k, b in enumerate(bs):
                b.out_len.zero_()
                b.ret.fill_(-1)
            torch.cuda.synchronize()
            for k, b in enumerate(bs):
                b.launch(ctx, dh, fl.root_type, 1, streams[k % 2].cuda_stream)
            torch.cuda.synchronize()
            got_r, got_o = [], []
            for b in bs:
                r, o = b.results()
                got_r += r
                got_o += o
            er, eo = _oracle_all(fl, msgs)
            assert got_r == er, rep
            assert got_o == eo, rep
    finally:
        ctx.close()


def test_many_streams_share_scratch_in_order():
    """More streams than the per-context scratch cap (8): shared scratches
    order the launches with events; results stay exact."""
    import torch
    fl = T.flatten(W.nesting_i64_desc())
    msgs = W.gen_nested_batch(random.Random(8), 12 * 200)
    ctx = conv.Context(0)
    try:
        dh = ctx.desc(fl)
        bs = [DevBatch(msgs[i:i + 200]) for i in range(0, len(msgs), 200)]
        streams = [torch.cuda.Stream() for _ in bs]
        torch.cuda.synchronize()
        for b, s in zip(bs, streams):
            b.launch(ctx, dh, fl.root_type, 1, s.cuda_stream)
        torch.cuda.synchronize()
        got_r, got_o = [], []
        for b in bs:
            r, o = b.results()
            got_r += r
            got_o += o
        er, eo = _oracle_all(fl, msgs)
        assert got_r == er and got_o == eo
    finally:
        ctx.close()


def test_desc_create_device_vs_oracle():
    """dg_desc_create_device: the blob arrives in device memory (as after an
    RCCL broadcast) and converts exactly like a host-created descriptor."""
    import torch
    fl = T.flatten(W.nesting_i64_desc())
    d_blob = torch.frombuffer(bytearray(fl.blob), dtype=torch.uint8).to("cuda:0")
    ctx = conv.Context(0)
    try:
        h = C.c_void_p()
        _lib.check(_lib.lib().dg_desc_create_device(ctx.h, d_blob.data_ptr(), d_blob.numel(), C.byref(h)))
        assert _lib.lib().dg_desc_root(h) == fl.root_type
        del d_blob  # the context keeps its own copy
        torch.cuda.synchronize()
        msgs = W.gen_nested_batch(random.Random(12), 1500) + [b"{}", b'{"I64":1', b""]
        b = DevBatch(msgs)
        s = torch.cuda.current_stream()
        b.launch(ctx, h, fl.root_type, 1, s.cuda_stream)
        torch.cuda.synchronize()
        r, o = b.results()
        er, eo = _oracle_all(fl, msgs)
        assert r == er and o == eo
        _lib.lib().dg_desc_destroy(h)
        # a corrupt device blob is refused
        bad = torch.zeros(64, dtype=torch.uint8, device="cuda:0")
        rc = _lib.lib().dg_desc_create_device(ctx.h, bad.data_ptr(), 64, C.byref(C.c_void_p()))
        assert rc == -4
    finally:
        ctx.close()


def test_overflow_needs_more_than_24_bits():
    """A message whose Thrift output exceeds 16 MiB overflows its default
    slot; the bytes needed travel in out_len (the 24-bit value field would
    truncate them) and the host entry point reruns it exactly."""
    td = T.list_of(T.struct_type("Wide", [T.FieldDescriptor(i, "f%d" % i, T.builtin("i64"), T.DEFAULT)
                                          for i in range(1, 400)]))
    fl = T.flatten(td)
    # each "{}" becomes 399 * 11 + 1 = 4390 bytes under WriteDefaultField
    m = b"[" + b",".join([b"{}"] * 4000) + b"]"  # ~17.6 MB of Thrift from 12 KB of JSON
    cv = conv.BinaryConv(conv.Options(WriteDefaultField=True))
    out = cv.do(fl, m)
    er, eo = _checker().j2t(fl, m, conv.to_flags(cv.opts))
    assert er == 0 and out == eo and len(out) > (1 << 24)


@pytest.mark.parametrize("n", [1, 300, 5000, 70001])
def test_pack_device_scan_vs_oracle(n):
    """dg_pack_device_scan: prefix sum of out_len + packing in one launch;
    the packed bytes are the oracle's outputs back to back (errors pack
    nothing), dst_off[n] is the total, nothing is written past it."""
    import torch
    rng = random.Random(n)
    msgs = W.gen_flat_batch(rng, n)
    for k in range(0, n, 97):
        msgs[k] = rng.choice([b"{]", b'{"I32Field":tru}', b"", b"{}", msgs[k]])
    fl = T.flatten(W.simple_desc())
    ctx = conv.default_context()
    b = DevBatch(msgs)
    s = torch.cuda.current_stream()
    b.launch(ctx, ctx.desc(fl), fl.root_type, 1, s.cuda_stream)
    d_dst = torch.full((int(b.slots[-1]) + 64,), 0xAB, dtype=torch.uint8, device="cuda:0")
    d_doff = torch.full((n + 1,), -1, dtype=torch.int64, device="cuda:0")
    for _ in range(2):  # twice: the arrival/departure counters self-reset
        _lib.check(_lib.lib().dg_pack_device_scan(ctx.h, b.out.data_ptr(), b.out_off.data_ptr(),
                                                  b.out_len.data_ptr(), n, d_dst.data_ptr(), d_doff.data_ptr(),
                                                  s.cuda_stream))
    torch.cuda.synchronize()
    er, eo = _oracle_all(fl, msgs)
    doff = d_doff.cpu().numpy()
    got = d_dst.cpu().numpy()
    want = b"".join(eo)
    assert int(doff[-1]) == len(want)
    assert got[:len(want)].tobytes() == want
    assert got[len(want)] == 0xAB
    exp_off = np.concatenate([[0], np.cumsum([len(o) for o in eo])])
    assert (doff == exp_off).all()


@pytest.mark.parametrize("cfg", ["c2", "c5mix"])
def test_batch_device_iters_vs_oracle(cfg):
    """dg_j2t_batch_device_iters (the bench's step loop): K back-to-back
    conversions of one batch leave exactly the oracle's output, on the flat
    path (C2) and on the small + wave + list pipeline (a C5-style mix)."""
    import torch
    rng = random.Random(77)
    if cfg == "c2":
        td, msgs = W.simple_desc(), W.gen_flat_batch(rng, 3000)
    else:
        td, msgs = W.mixed_desc(), W.gen_mixed_batch(rng, 1500, large_scale=0.05)
    fl = T.flatten(td)
    ctx = conv.default_context()
    dh = ctx.desc(fl)
    b = DevBatch(msgs)
    st = torch.cuda.current_stream().cuda_stream
    for ml in (0, b.max_len):
        b.out.zero_()
        b.ret.fill_(-1)
        _lib.check(_lib.lib().dg_j2t_batch_device_iters(
            ctx.h, dh, fl.root_type, b.json.data_ptr(), b.in_off.data_ptr(), b.n, 1, b.out.data_ptr(),
            b.out_off.data_ptr(), b.out_len.data_ptr(), b.ret.data_ptr(), None, st, ml, 3))
        torch.cuda.synchronize()
        assert b.results() == _oracle_all(fl, msgs)


@pytest.mark.parametrize("cfg", ["c2", "c5mix"])
@pytest.mark.parametrize("depth", [2, 3])
def test_batch_device_inflight_vs_oracle(cfg, depth):
    """dg_j2t_batch_device_inflight (the bench's timed steps): `depth`
    conversions in flight on the context's streams, each into its own output
    set; every set holds exactly the oracle's output, and work enqueued on the
    caller's stream afterwards sees all of them done (the join)."""
    import torch
    rng = random.Random(78)
    if cfg == "c2":
        td, msgs = W.simple_desc(), W.gen_flat_batch(rng, 3000)
    else:
        td, msgs = W.mixed_desc(), W.gen_mixed_batch(rng, 1500, large_scale=0.05)
    fl = T.flatten(td)
    ctx = conv.default_context()
    dh = ctx.desc(fl)
    bs = [DevBatch(msgs) for _ in range(depth)]
    pend = [torch.zeros(4, dtype=torch.int32, device="cuda:0") for _ in range(depth)]
    for b in bs:
        b.out.zero_()
        b.ret.fill_(-1)
    sets = (C.c_void_p * (4 * depth))(*[p for b, pd in zip(bs, pend)
                                          for p in (b.out.data_ptr(), b.out_len.data_ptr(), b.ret.data_ptr(),
                                                    pd.data_ptr())])
    s = torch.cuda.Stream()
    _lib.check(_lib.lib().dg_j2t_batch_device_inflight(
        ctx.h, dh, fl.root_type, bs[0].json.data_ptr(), bs[0].in_off.data_ptr(), bs[0].n, 1,
        bs[0].out_off.data_ptr(), sets, depth, s.cuda_stream, bs[0].max_len, 2 * depth + 1))
    # the join: copies enqueued on the caller's stream see every set finished
    with torch.cuda.stream(s):
        got = [(b.out.clone(), b.out_len.clone(), b.ret.clone()) for b in bs]
    s.synchronize()
    exp = _oracle_all(fl, msgs)
    for b, (o, ol, r) in zip(bs, got):
        b.out, b.out_len, b.ret = o, ol, r
        assert b.results() == exp
    assert all(int(p.sum().item()) == 0 for p in pend)
