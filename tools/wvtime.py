"""Time the default pipeline on C3 with whatever library DG_LIB_PATH names (ablation builds), no checks."""
import ctypes as C
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from dynamicgo_amd import _lib, conv, workloads as W
from dynamicgo_amd.thrift import flatten

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
td, msgs = W.nesting_i64_desc(), W.gen_nested_batch(random.Random(43), n)
flat = flatten(td)
a, off = W.arena(msgs)
slots = np.zeros(n + 1, dtype=np.int64)
np.cumsum((np.diff(off).astype(np.int64) * 4 + 64 + 7) // 8 * 8, out=slots[1:])
dev = torch.device("cuda:0")
ctx = conv.Context(0)
dh = ctx.desc(flat)
d_json = torch.from_numpy(a).to(dev)
d_in = torch.from_numpy(off.astype(np.int64)).to(dev)
d_out = torch.empty(int(slots[-1]) + 64, dtype=torch.uint8, device=dev)
d_oo = torch.from_numpy(slots).to(dev)
d_ol = torch.zeros(n, dtype=torch.int32, device=dev)
d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
L = _lib.lib()
ms = C.c_float(0)
args = (ctx.h, dh, flat.root_type, d_json.data_ptr(), d_in.data_ptr(), n, 1, d_out.data_ptr(), d_oo.data_ptr(),
        d_ol.data_ptr(), d_ret.data_ptr())
_lib.check(L.dg_bench_device(*args, 2, C.byref(ms)))
best = 1e9
for _ in range(3):
    _lib.check(L.dg_bench_device(*args, 5, C.byref(ms)))
    best = min(best, ms.value / 5)
print(f"{os.environ.get('DG_LIB_PATH', 'libdgj2t.so')} c3: {best * 1000:.1f} us/step ok={(d_ret.cpu().numpy() == 0).sum()}")
