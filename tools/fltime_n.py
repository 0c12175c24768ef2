"""Time the C2 pipeline (flat kernel + list pass) at several batch sizes: is
the step time set by the number of block rounds? python tools/fltime_n.py"""
import ctypes as C
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from dynamicgo_amd import _lib, conv, workloads as W
from dynamicgo_amd.thrift import flatten

msgs_all = W.gen_flat_batch(random.Random(42), 65536)
flat = flatten(W.simple_desc())
dev = torch.device("cuda:0")
ctx = conv.Context(0)
dh = ctx.desc(flat)
L = _lib.lib()
for n in ([int(x) for x in sys.argv[1:]] or (12288, 24576, 36864, 49152, 57344, 65536)):
    msgs = msgs_all[:n]
    a, off = W.arena(msgs)
    slots = np.zeros(n + 1, dtype=np.int64)
    np.cumsum((np.diff(off).astype(np.int64) * 4 + 64 + 7) // 8 * 8, out=slots[1:])
    d_json = torch.from_numpy(a).to(dev)
    d_in = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_out = torch.empty(int(slots[-1]) + 64, dtype=torch.uint8, device=dev)
    d_oo = torch.from_numpy(slots).to(dev)
    d_ol = torch.zeros(n, dtype=torch.int32, device=dev)
    d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
    s = torch.cuda.Stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    args = (ctx.h, dh, flat.root_type, d_json.data_ptr(), d_in.data_ptr(), n, 1, d_out.data_ptr(), d_oo.data_ptr(),
            d_ol.data_ptr(), d_ret.data_ptr(), None, s.cuda_stream, 256)
    _lib.check(L.dg_j2t_batch_device_iters(*args, 5))
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0.record(s)
        _lib.check(L.dg_j2t_batch_device_iters(*args, 20))
        e1.record(s)
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 20)
    print(f"n={n} blocks={n // 64} {best * 1000:.1f} us/step ok={(d_ret.cpu().numpy() == 0).sum()}", flush=True)
