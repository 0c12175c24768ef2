"""Phase breakdown of the wave kernel (a -DDG_WPROF build, DG_LIB_PATH) on a
bench config: python tools/wprof.py c3 [n]"""
import os, sys, random
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import ctypes as C
from dynamicgo_amd import _lib, conv, workloads as W
from dynamicgo_amd.thrift import flatten

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
gen = {"c2": (W.simple_desc, lambda r, k: W.gen_flat_batch(r, k), 42),
       "c3": (W.nesting_i64_desc, lambda r, k: W.gen_nested_batch(r, k), 43),
       "c4": (W.large_desc, lambda r, k: W.gen_large_batch(r, k), 44)}[cfg]
td, msgs = gen[0](), gen[1](random.Random(gen[2]), n)
flat = flatten(td)
a, off = W.arena(msgs)
slots = np.zeros(n + 1, dtype=np.int64)
np.cumsum((np.diff(off).astype(np.int64) * 4 + 64 + 7) // 8 * 8, out=slots[1:])
dev = torch.device("cuda:0")
ctx = conv.Context(0)
dh = ctx.desc(flat)
d_json = torch.from_numpy(a).to(dev); d_in = torch.from_numpy(off.astype(np.int64)).to(dev)
d_out = torch.empty(int(slots[-1]) + 64, dtype=torch.uint8, device=dev); d_oo = torch.from_numpy(slots).to(dev)
d_ol = torch.zeros(n, dtype=torch.int32, device=dev); d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
L = _lib.lib()
ms = C.c_float(0)
cnt = (C.c_uint64 * 16)()
for it in (1, 5):
    _lib.check(L.dg_ctx_counters(ctx.h, cnt, 16, 1))
    _lib.check(L.dg_bench_device(ctx.h, dh, flat.root_type, d_json.data_ptr(), d_in.data_ptr(), n, 1, d_out.data_ptr(),
                                 d_oo.data_ptr(), d_ol.data_ptr(), d_ret.data_ptr(), it, C.byref(ms)))
_lib.check(L.dg_ctx_counters(ctx.h, cnt, 16, 1))
c = list(cnt)
names = ["scan", "depth/grammar", "parent+ctx", "types", "len A", "len B", "offsets+emit", "long str", "stack", "-"]
tot = sum(c[2:12])
print(f"{cfg}: {ms.value / 5 * 1000:.1f} us/step, bails/step {c[0] / 5:.1f}, ok={(d_ret.cpu().numpy() == 0).sum()}")
for k, nm in enumerate(names):
    print("  %-16s %6.2f%%  %10.0f cycles/msg" % (nm, 100 * c[2 + k] / max(1, tot), c[2 + k] / 5 / n))
