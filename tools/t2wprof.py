"""Phase breakdown of the t2j wave kernel (a -DDG_T2W_PROF build via
DG_LIB_PATH) on t2j-c3: python tools/t2wprof.py [n]"""
import ctypes as C
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from dynamicgo_amd import _lib, conv, t2j, workloads as W
from dynamicgo_amd.thrift import flatten

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
td = W.nesting_i64_desc()
fl = flatten(td)
thr, rets = conv.BinaryConv(conv.Options()).do_batch(td, W.gen_nested_batch(random.Random(43), n))
a, off = W.arena(thr)
tl = np.diff(off).astype(np.int64)
jo = np.zeros(n + 1, dtype=np.int64)
np.cumsum((tl * 3 + 64 + 7) // 8 * 8, out=jo[1:])
dev = torch.device("cuda:0")
ctx = conv.Context(0)
dh = ctx.desc_t2j(fl)
d_src = torch.from_numpy(a).to(dev)
d_in = torch.from_numpy(off.astype(np.int64)).to(dev)
d_out = torch.empty(int(jo[-1]) + 64, dtype=torch.uint8, device=dev)
d_jo = torch.from_numpy(jo).to(dev)
d_jl = torch.zeros(n, dtype=torch.int32, device=dev)
d_jr = torch.zeros(n, dtype=torch.int64, device=dev)
L = _lib.lib()
cnt = (C.c_uint64 * 16)()
s = torch.cuda.current_stream()
for it in range(3):
    _lib.check(L.dg_ctx_counters(ctx.h, cnt, 16, 1))
    _lib.check(L.dg_t2j_batch_device_ml(ctx.h, dh, fl.root_type, d_src.data_ptr(), d_in.data_ptr(), n, 0,
                                        d_out.data_ptr(), d_jo.data_ptr(), d_jl.data_ptr(), d_jr.data_ptr(),
                                        s.cuda_stream, int(tl.max())))
    torch.cuda.synchronize()
_lib.check(L.dg_ctx_counters(ctx.h, cnt, 16, 1))
c = list(cnt)
names = ["walk (all lanes)", "tok+esc scan", "numbers", "len+prefix+write", "stage+other", "copy tasks"]
tot = sum(c[2:8])
print(f"ok={(d_jr.cpu().numpy() == 0).sum()} of {n}")
for k, nm in enumerate(names):
    print("  %-12s %6.2f%%  %10.0f cycles/msg" % (nm, 100 * c[2 + k] / max(1, tot), c[2 + k] / n))
