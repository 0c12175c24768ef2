"""Debug: the concurrent blocking-Do aggregator case, with the differing
calls printed (index, message kind, expected vs got status and lengths)."""
import os, random, sys, threading
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import oracle
from dynamicgo_amd import conv, thrift as T, workloads as W

def run(errors: bool, nthreads: int, max_batch: int):
    td = W.nesting_i64_desc()
    rng = random.Random(3)
    msgs = W.gen_nested_batch(rng, 1200) + ([b"{]", b"", b"null", b'{"I64":"x"}'] * 10 if errors else [])
    rng.shuffle(msgs)
    fl = T.flatten(td)
    chk = oracle.RefOracle() or oracle.PortOracle()
    want = [chk.j2t(fl, m, 1) for m in msgs]
    agg = conv.Aggregator(td, conv.Options(), max_batch=max_batch, max_wait_us=2000)
    got = [None] * len(msgs)
    def worker(k):
        for i in range(k, len(msgs), nthreads):
            try:
                got[i] = (0, agg.do(msgs[i]) or b"")
            except conv.J2TError as e:
                got[i] = (e.ret, b"")
    ths = [threading.Thread(target=worker, args=(k,)) for k in range(nthreads)]
    for t in ths: t.start()
    for t in ths: t.join(timeout=120)
    batches, n = agg.stats()
    prof = agg.profile()
    agg.close()
    bad = [i for i in range(len(msgs)) if got[i] != tuple(want[i])]
    print(f"errors={errors} threads={nthreads} max_batch={max_batch}: batches={batches} n={n} bad={len(bad)} fallback={prof[11]}")
    for i in bad[:8]:
        g, w = got[i], want[i]
        print("  ", i, len(msgs[i]), msgs[i][:20], "thread", i % nthreads, "got", hex(g[0]) if g else None, len(g[1]) if g else None,
              "want", hex(w[0]), len(w[1]), "first diff", next((k for k in range(min(len(g[1]), len(w[1]))) if g[1][k] != w[1][k]), None) if g else None)
    return len(bad)

if __name__ == "__main__":
    tot = 0
    for rep in range(int(os.environ.get("REPS", "12"))):
        tot += run(True, 16, 256)
    print("total bad", tot)
