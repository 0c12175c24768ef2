import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "tests")); sys.path.insert(0, os.path.join(R, "oracle"))
import oracle
from dynamicgo_amd import thrift as T, workloads as W
from test_gpu_parity import _raw_batch
chk = oracle.RefOracle() or oracle.PortOracle()
for dn in ("nesting_i64_desc", "nesting_desc", "mixed_desc", "simple_desc"):
    fl = T.flatten(getattr(W, dn)())
    msgs = [b'{}', b'{"I32":5}', b'{"Nested":{}}']
    for flags in (0x7, 0x5, 0x3, 0x6):
        outs, rets = _raw_batch(fl, msgs, flags)
        er, eo = chk.j2t_batch(fl, msgs, flags)
        for i, m in enumerate(msgs):
            if outs[i] != eo[i] or int(rets[i]) != int(er[i]):
                print(dn, hex(flags), m, "GPU", len(outs[i]), outs[i][:80].hex(), "\n   REF", len(eo[i]), eo[i][:80].hex())
                break
