"""The batching aggregator (dg_agg): many threads
calling Do concurrently, like the reference's RunParallel benchmark
(conv/j2t/conv_timing_test.go:76-99), get the oracle's bytes and status
words, and their calls are coalesced into device batches."""
import random
import threading

import pytest

import oracle
from dynamicgo_amd import conv, thrift as T, workloads as W

pytestmark = pytest.mark.gpu


def test_aggregator_concurrent_do_vs_oracle():
    td = W.nesting_i64_desc()
    rng = random.Random(3)
    msgs = W.gen_nested_batch(rng, 1200) + [b"{]", b"", b"null", b'{"I64":"x"}'] * 10
    rng.shuffle(msgs)
    fl = T.flatten(td)
    chk = oracle.RefOracle() or oracle.PortOracle()
    want = [chk.j2t(fl, m, 1) for m in msgs]
    agg = conv.Aggregator(td, conv.Options(), max_batch=256, max_wait_us=2000)
    got = [None] * len(msgs)

    def worker(k):
        for i in range(k, len(msgs), 16):
            try:
                got[i] = (0, agg.do(msgs[i]) or b"")
            except conv.J2TError as e:
                got[i] = (e.ret, b"")

    ths = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    batches, n = agg.stats()
    agg.close()
    assert n == len(msgs)
    # coalesced, not one launch per call: a batch is sealed once every thread
    # with a call in it is blocked on it
    assert batches < len(msgs) // 2, batches
    assert got == [(r, o) for r, o in want]


def test_aggregator_grows_output_and_drains_on_close():
    fields = [T.FieldDescriptor(i, "f%d" % i, T.builtin("i64"), T.DEFAULT) for i in range(1, 200)]
    td = T.struct_type("Wide", fields)
    agg = conv.Aggregator(td, conv.Options(WriteDefaultField=True), max_batch=8, max_wait_us=100)
    out = agg.do(b"{}")  # 2 bytes of JSON -> 2190 bytes of Thrift: the retry path
    chk = oracle.RefOracle() or oracle.PortOracle()
    assert out == chk.j2t(T.flatten(td), b"{}", 0x3)[1]
    agg.close()


def _mixed_msgs(n, seed):
    rng = random.Random(seed)
    msgs = W.gen_nested_batch(rng, n) + [b"{]", b"", b"null", b'{"I64":"x"}'] * 8
    rng.shuffle(msgs)
    return msgs


@pytest.mark.parametrize("threads,window,max_batch", [(8, 64, 128), (16, 300, 1024), (3, 1, 64)])
def test_aggregator_drive_vs_oracle(threads, window, max_batch):
    """dg_agg_drive: many threads with many calls in flight each (the async
    submit/wait form); small batches force the ring of in-flight batches to
    wrap many times and callers to meet sealed batches."""
    td = W.nesting_i64_desc()
    msgs = _mixed_msgs(3000, 11)
    fl = T.flatten(td)
    chk = oracle.RefOracle() or oracle.PortOracle()
    want = [chk.j2t(fl, m, 1) for m in msgs]
    agg = conv.Aggregator(td, conv.Options(), max_batch=max_batch, max_wait_us=500, max_bytes=max_batch * 1200)
    outs, rets, lat, secs = agg.drive(msgs, threads=threads, window=window)
    batches, n = agg.stats()
    agg.close()
    assert n == len(msgs)
    assert batches >= len(msgs) // (max_batch * threads)  # max_batch: per thread and batch
    assert [(int(r), o if int(r) == 0 else b"") for r, o in zip(rets, outs)] == \
        [(r, o if r == 0 else b"") for r, o in want]
    assert secs > 0 and int(lat.max()) > 0


def test_aggregator_byte_capacity_and_oversize():
    """A batch sealed by its JSON capacity (not its count), and a message
    longer than a whole batch (converted alone)."""
    td = W.nesting_i64_desc()
    rng = random.Random(5)
    msgs = W.gen_nested_batch(rng, 400)
    big = max(msgs, key=len)
    msgs = msgs + [big]
    fl = T.flatten(td)
    chk = oracle.RefOracle() or oracle.PortOracle()
    want = [chk.j2t(fl, m, 1) for m in msgs]
    agg = conv.Aggregator(td, conv.Options(), max_batch=4096, max_wait_us=300, max_bytes=len(big) * 3 - 1)
    outs, rets, _, _ = agg.drive(msgs, threads=4, window=32)
    agg.close()
    assert [(int(r), o) for r, o in zip(rets, outs)] == [(r, o) for r, o in want]
    agg = conv.Aggregator(td, conv.Options(), max_batch=64, max_wait_us=300, max_bytes=len(big) - 1)
    assert agg.do(big) == want[-1][1]
    agg.close()


@pytest.mark.parametrize("chunks", [1, 3, 7])
def test_pipeline_host_vs_oracle(chunks):
    """dg_j2t_pipeline_host: the same outputs as dg_j2t_batch_host and the
    oracle, for any chunking."""
    td = W.nesting_i64_desc()
    msgs = _mixed_msgs(2500, 12)
    fl = T.flatten(td)
    chk = oracle.RefOracle() or oracle.PortOracle()
    want = [chk.j2t(fl, m, 1) for m in msgs]
    cv = conv.BinaryConv(conv.Options())
    outs, rets = cv.do_batch(td, msgs, chunks=chunks)
    assert [(int(r), o if int(r) == 0 else b"") for r, o in zip(rets, outs)] == \
        [(r, o if r == 0 else b"") for r, o in want]


def test_pipeline_host_overflow_splice_and_nomem():
    """Slot overflows (2 bytes of JSON -> 2190 bytes of Thrift) are rerun and
    spliced in place, in every chunk; a too-small out_cap gives DG_E_NOMEM
    with the exact need, and the retry succeeds."""
    fields = [T.FieldDescriptor(i, "f%d" % i, T.builtin("i64"), T.DEFAULT) for i in range(1, 200)]
    td = T.struct_type("Wide", fields)
    rng = random.Random(9)
    msgs = []
    for i in range(900):
        if rng.random() < 0.05:
            msgs.append(b"{}")
        else:
            ks = rng.sample(range(1, 200), 150)
            msgs.append(("{" + ",".join('"f%d":%d' % (k, rng.randrange(-10**12, 10**12)) for k in ks) + "}").encode())
    fl = T.flatten(td)
    chk = oracle.RefOracle() or oracle.PortOracle()
    opts = conv.Options(WriteDefaultField=True)
    want = [chk.j2t(fl, m, conv.to_flags(opts)) for m in msgs]
    cv = conv.BinaryConv(opts)
    for chunks in (1, 4):
        outs, rets = cv.do_batch(td, msgs, chunks=chunks)
        assert [(int(r), o) for r, o in zip(rets, outs)] == [(r, o) for r, o in want]
    outs, rets = cv.do_batch(td, msgs, chunks=3, out_cap=1000)  # NOMEM first, then the exact need
    assert [(int(r), o) for r, o in zip(rets, outs)] == [(r, o) for r, o in want]


@pytest.mark.parametrize("chunks,shift,jshift", [(1, 0, 0), (5, 0, 0), (1, 3, 0), (4, 11, 0), (1, 0, 5), (3, 2, 8)])
def test_pipeline_host_pinned_direct(chunks, shift, jshift):
    """With pinned host buffers the chained packing writes the caller's
    out / out_off straight from the GPU; a too-small out_cap writes nothing
    past it and reports the exact need. shift: `out` starts that many bytes
    into a pinned allocation (not 16-aligned: the first chunk's copy-out
    must not drop its bytes). jshift: the JSON arena starts that many bytes
    into a pinned allocation (not 16-aligned, so the kernels must
    not read it in place with 16-byte loads; the staged copy is used)."""
    import ctypes as C
    import numpy as np
    import torch
    from dynamicgo_amd import _lib
    td = W.nesting_i64_desc()
    msgs = _mixed_msgs(1500, 13)
    fl = T.flatten(td)
    chk = oracle.RefOracle() or oracle.PortOracle()
    want = [chk.j2t(fl, m, 1) for m in msgs]
    n = len(msgs)
    a, off = W.arena(msgs)
    h_jbuf = torch.zeros(len(a) + jshift, dtype=torch.uint8).pin_memory()
    h_jbuf[jshift:] = torch.from_numpy(a)
    h_json = h_jbuf[jshift:]
    h_in = torch.from_numpy(off.astype(np.int64)).pin_memory()
    cv = conv.BinaryConv(conv.Options())
    ctx = cv._ctx()
    L = _lib.lib()
    need = C.c_uint64(0)
    for cap in (1000, int(off[-1]) * 4 + 80 * n + 64):
        h_buf = torch.full((cap + 64 + shift,), 0xAB, dtype=torch.uint8).pin_memory()
        h_out = h_buf[shift:]
        h_oo = torch.zeros(n + 1, dtype=torch.int64).pin_memory()
        h_ret = torch.zeros(n, dtype=torch.int64).pin_memory()
        rc = L.dg_j2t_pipeline_host(ctx.h, ctx.desc(fl), fl.root_type, h_json.data_ptr(), h_in.data_ptr(), n, 1,
                                    chunks, h_out.data_ptr(), cap, h_oo.data_ptr(), h_ret.data_ptr(), C.byref(need))
        tail = h_out.numpy()[cap:]
        assert (tail == 0xAB).all()  # nothing written past out_cap
        if cap == 1000:
            assert rc == -3 and need.value > cap
            continue
        _lib.check(rc)
        ob, oo, rr = h_out.numpy(), h_oo.numpy(), h_ret.numpy()
        assert int(oo[-1]) == need.value
        got = [(int(rr[i]), ob[oo[i]:oo[i + 1]].tobytes()) for i in range(n)]
        assert got == [(r, o if r == 0 else b"") for r, o in want]


def test_aggregator_parts_return_at_thread_exit():
    """400 short-lived threads (more than the 256 parts), each one
    blocking Do: an exited thread's part goes to the next thread, so no call
    falls back to the unbatched path, and every result is the oracle's."""
    td = W.nesting_i64_desc()
    fl = T.flatten(td)
    msgs = W.gen_nested_batch(random.Random(8), 400)
    chk = oracle.RefOracle() or oracle.PortOracle()
    agg = conv.Aggregator(td, conv.Options(), max_batch=64, max_wait_us=50)
    got = [None] * len(msgs)

    def one(i):
        got[i] = agg.do(msgs[i]) or b""

    for k in range(0, len(msgs), 8):  # 8 at a time, each thread gone before the next wave
        ths = [threading.Thread(target=one, args=(i,)) for i in range(k, min(k + 8, len(msgs)))]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=60)
    prof = agg.profile()
    agg.close()
    assert prof[11] == 0, prof
    assert got == [chk.j2t(fl, m, 1)[1] for m in msgs]


def test_aggregator_fresh_contexts_first_batches():
    """The first batches on a fresh context's streams: the per-stream list
    counters must be zero before the aggregator's non-blocking streams use
    them (a null-stream hipMemset was not ordered before those launches, and
    the first batches left some messages unconverted: ret 0, no bytes)."""
    td = W.nesting_i64_desc()
    fl = T.flatten(td)
    chk = oracle.RefOracle() or oracle.PortOracle()
    msgs = W.gen_nested_batch(random.Random(9), 600)
    want = [chk.j2t(fl, m, 1)[1] for m in msgs]
    for rep in range(3):
        ctx = conv.Context(0)
        agg = conv.Aggregator(td, conv.Options(), max_batch=64, max_wait_us=200, ctx=ctx)
        outs, rets, _, _ = agg.drive(msgs, threads=16, window=16)
        agg.close()
        assert [int(r) for r in rets] == [0] * len(msgs)
        assert outs == want, rep


@pytest.mark.parametrize("callers,workers,depth,fill", [(1024, 8, 2, 0), (4096, 16, 3, 512), (5, 3, 0, 0), (300, 2, 1, 64)])
def test_gateway_drive_vs_oracle(callers, workers, depth, fill):
    """The gateway shape: many logical callers with ONE call
    in flight each (goroutines in Do), multiplexed over a few OS threads and
    woken per converted generation by one dg_agg_wait_gen poller -- no OS
    thread blocks per call. Every result is the oracle's."""
    td = W.nesting_i64_desc()
    msgs = _mixed_msgs(6000, 21)
    fl = T.flatten(td)
    chk = oracle.RefOracle() or oracle.PortOracle()
    want = [chk.j2t(fl, m, 1) for m in msgs]
    agg = conv.Aggregator(td, conv.Options(), max_batch=512, max_wait_us=300, max_bytes=512 * 3000)
    if depth:
        agg.set_knob("depth", depth)
    if fill:
        agg.set_knob("min_fill", fill)
    outs, rets, lat, secs, st = agg.gateway(msgs, callers=callers, workers=workers)
    batches, n = agg.stats()
    prof = agg.profile()
    agg.close()
    assert n == len(msgs) and prof[11] == 0
    assert st[3] == min(callers, len(msgs)) and st[7] > 0
    assert [(int(r), o if int(r) == 0 else b"") for r, o in zip(rets, outs)] == \
        [(r, o if r == 0 else b"") for r, o in want]
    assert secs > 0 and int(lat.max()) > 0


@pytest.mark.parametrize("n,callers,workers", [(10, 64, 16), (600, 3, 16), (2, 1, 16)])
def test_gateway_drive_fewer_callers_or_messages_than_workers(n, callers, workers):
    """worker w owns messages [n w / W, n (w+1) / W) but only the
    callers c = w (mod W); with fewer callers (or messages) than workers some
    workers owned messages no caller submitted and the drive never ended.
    Workers are clamped to min(workers, callers, n); every result is the
    oracle's."""
    td = W.nesting_i64_desc()
    msgs = W.gen_nested_batch(random.Random(23), n)
    fl = T.flatten(td)
    chk = oracle.RefOracle() or oracle.PortOracle()
    want = [chk.j2t(fl, m, 1) for m in msgs]
    agg = conv.Aggregator(td, conv.Options(), max_batch=256, max_wait_us=200, max_bytes=512 * 3000)
    outs, rets, lat, secs, st = agg.gateway(msgs, callers=callers, workers=workers)
    agg.close()
    assert st[3] == min(callers, n)
    assert [(int(r), o if int(r) == 0 else b"") for r, o in zip(rets, outs)] == \
        [(r, o if r == 0 else b"") for r, o in want]


def test_aggregator_shared_parts_past_224_threads():
    """More concurrent threads than exclusive parts: threads 225+ share the
    last 32 parts under their lock instead of converting alone (the r4
    256-thread cliff), and every result is the oracle's."""
    td = W.nesting_i64_desc()
    fl = T.flatten(td)
    msgs = W.gen_nested_batch(random.Random(31), 900)
    chk = oracle.RefOracle() or oracle.PortOracle()
    want = [chk.j2t(fl, m, 1)[1] for m in msgs]
    agg = conv.Aggregator(td, conv.Options(), max_batch=16, max_wait_us=200, max_bytes=64 * 1024)
    got = [None] * len(msgs)
    go = threading.Event()

    def worker(k):
        go.wait()
        for i in range(k, len(msgs), 300):
            got[i] = agg.do(msgs[i]) or b""

    ths = [threading.Thread(target=worker, args=(k,)) for k in range(300)]
    for t in ths:
        t.start()
    go.set()
    for t in ths:
        t.join(timeout=120)
    prof = agg.profile()
    agg.close()
    assert prof[11] == 0, prof
    assert got == want
