"""Repro of a fuzz mismatch on schemas.probe('D3') (flags 0x23) over every route."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, "tests")
sys.path.insert(0, "tests/golden")
sys.path.insert(0, "oracle")
import oracle
from dynamicgo_amd import thrift as T
from schemas import probe
from test_gpu_parity import _raw_batch

m = (b'{"0A":\r\nnull,"A":\t  256,"B":"\\ud83d\\ude00\\n\xe4\xb8\xad\xe6\x96\x87\\u00e9\xe4\xb8\xad\xe6\x96\x87')
fl = T.flatten(probe("D3"))
chk = oracle.RefOracle() or oracle.PortOracle()
print("expected", hex(chk.j2t(fl, m, 0x23)[0]), len(m))
for name, fx in [("default", 0), ("no_flat", 1 << 21), ("flat", 1 << 19), ("no_wave", 1 << 18), ("no_fast", 1 << 17)]:
    outs, rets = _raw_batch(fl, [m], 0x23 | fx)
    print(name, hex(int(rets[0])))
    outs, rets = _raw_batch(fl, [m, b'{"A":' + b'1' * 600 + b'}'], 0x23 | fx)
    print(name, "+big", hex(int(rets[0])))

import random
import fuzz
td = probe("D3")
nbad = 0
for seed in range(40):
    rng = random.Random(seed)
    msgs = [fuzz.gen_message(rng, td, mutate_p=rng.random() < 0.5) for _ in range(300)]
    outs, rets = _raw_batch(fl, msgs, 0x23)
    for mm, o, r in zip(msgs, outs, rets):
        er, eo = chk.j2t(fl, mm, 0x23)
        if (int(r), o) != (er, eo):
            nbad += 1
            if nbad <= 3:
                print("seed", seed, "len", len(mm), hex(int(r)), hex(er), mm[:200])
print("mismatches", nbad)
