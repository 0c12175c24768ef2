"""C2 throughput with successive batches alternating over S streams (each
stream its own output buffers; the library keeps per-stream scratch):
python tools/twostream.py [S] [steps]"""
import os, random, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from dynamicgo_amd import _lib, conv, workloads as W
from dynamicgo_amd.thrift import flatten

S = int(sys.argv[1]) if len(sys.argv) > 1 else 2
K = int(sys.argv[2]) if len(sys.argv) > 2 else 40
td = W.simple_desc()
msgs = W.gen_flat_batch(random.Random(42), 65536)
a, off = W.arena(msgs)
n = len(msgs)
fl = flatten(td)
dev = torch.device("cuda:0")
ctx = conv.Context(0)
dh = ctx.desc(fl)
L = _lib.lib()
lens = np.diff(off).astype(np.int64)
slots = np.zeros(n + 1, dtype=np.int64)
np.cumsum((lens * 4 + 64 + 7) & ~7, out=slots[1:])
d_json = torch.from_numpy(a).to(dev)
d_in = torch.from_numpy(off.astype(np.int64)).to(dev)
d_oo = torch.from_numpy(slots).to(dev)
sets = []
for k in range(S):
    sets.append(dict(out=torch.empty(int(slots[-1]) + 64, dtype=torch.uint8, device=dev),
                     ol=torch.zeros(n, dtype=torch.int32, device=dev), ret=torch.zeros(n, dtype=torch.int64, device=dev),
                     pend=torch.zeros(4, dtype=torch.int32, device=dev), st=torch.cuda.Stream(dev)))
ml = int(lens.max())


def step(k):
    z = sets[k % S]
    _lib.check(L.dg_j2t_batch_device_iters(ctx.h, dh, fl.root_type, d_json.data_ptr(), d_in.data_ptr(), n, 1,
                                           z["out"].data_ptr(), d_oo.data_ptr(), z["ol"].data_ptr(), z["ret"].data_ptr(),
                                           z["pend"].data_ptr(), z["st"].cuda_stream, ml, 1))


for k in range(10):
    step(k)
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    for k in range(K):
        step(k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"S={S}: {dt / K * 1e6:.1f} us/step, {int(off[-1]) * K / dt / 1e9:.1f} GB/s", flush=True)
print("ok", all(int((z["ret"] != 0).sum()) == 0 for z in sets))
