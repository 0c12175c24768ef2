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
    assert batches < len(msgs) // 4, batches  # coalesced, not one launch per call
    assert got == [(r, o) for r, o in want]


def test_aggregator_grows_output_and_drains_on_close():
    fields = [T.FieldDescriptor(i, "f%d" % i, T.builtin("i64"), T.DEFAULT) for i in range(1, 200)]
    td = T.struct_type("Wide", fields)
    agg = conv.Aggregator(td, conv.Options(WriteDefaultField=True), max_batch=8, max_wait_us=100)
    out = agg.do(b"{}")  # 2 bytes of JSON -> 2190 bytes of Thrift: the retry path
    chk = oracle.RefOracle() or oracle.PortOracle()
    assert out == chk.j2t(T.flatten(td), b"{}", 0x3)[1]
    agg.close()
