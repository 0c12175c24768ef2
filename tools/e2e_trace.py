"""Drive dg_j2t_pipeline_host on C2 with pinned buffers (for a rocprofv3
timeline), and time CPU reads/writes of pinned vs pageable host memory:
python tools/e2e_trace.py [chunks] [reps]"""
import ctypes as C
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from dynamicgo_amd import _lib, conv, workloads as W
from dynamicgo_amd.thrift import flatten

chunks = int(sys.argv[1]) if len(sys.argv) > 1 else 4
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
td = W.simple_desc()
msgs = W.gen_flat_batch(random.Random(42), 65536)
a, off = W.arena(msgs)
n = len(msgs)
fl = flatten(td)
ctx = conv.Context(0)
L = _lib.lib()
h_json = torch.from_numpy(a).pin_memory()
h_in = torch.from_numpy(off.astype(np.int64)).pin_memory()
cap = int(off[-1]) * 4 + 80 * n + 64
h_out = torch.empty(cap, dtype=torch.uint8).pin_memory()
h_oo = torch.zeros(n + 1, dtype=torch.int64).pin_memory()
h_ret = torch.zeros(n, dtype=torch.int64).pin_memory()
need = C.c_uint64(0)
for k in [1, chunks] + [chunks] * reps:
    t0 = time.perf_counter()
    _lib.check(L.dg_j2t_pipeline_host(ctx.h, ctx.desc(fl), fl.root_type, h_json.data_ptr(), h_in.data_ptr(), n, 1, k,
                                      h_out.data_ptr(), cap, h_oo.data_ptr(), h_ret.data_ptr(), C.byref(need)))
    print(f"chunks={k}: {(time.perf_counter() - t0) * 1e3:.3f} ms", flush=True)
# CPU access to pinned host memory vs pageable
for name, buf in (("pinned", torch.empty(16 << 20, dtype=torch.uint8).pin_memory()),
                  ("pageable", torch.empty(16 << 20, dtype=torch.uint8))):
    x = buf.numpy()
    src = np.random.randint(0, 255, 16 << 20, dtype=np.uint8)
    t0 = time.perf_counter(); x[:] = src; tw = time.perf_counter() - t0
    t0 = time.perf_counter(); y = x.copy(); tr = time.perf_counter() - t0
    t0 = time.perf_counter(); s = int(x[::64].sum()); tl = time.perf_counter() - t0
    print(f"{name}: write {16 / tw / 1024:.2f} GB/s, read {16 / tr / 1024:.2f} GB/s, strided 64 B reads "
          f"{tl / (len(x) // 64) * 1e9:.1f} ns each", flush=True)
