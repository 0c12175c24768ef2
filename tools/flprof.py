"""Phase breakdown of the flat kernel (a -DDG_FLPROF build, tools/build_variants.py flprof=-DDG_FL_PROF...):
on the GPU: DG_LIB_PATH=dynamicgo_amd/libdgj2t_flprof.so DG_ALLOW_STALE=1 python tools/flprof.py c2"""
import ctypes as C
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from dynamicgo_amd import _lib, conv, workloads as W
from dynamicgo_amd.thrift import flatten

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
fields = "--fields" in sys.argv  # a -DDG_FLPROF_F build: per field slot parse / write cycles
td, msgs = {"c2": lambda: (W.simple_desc(), W.gen_flat_batch(random.Random(42), 65536)),
            "c2s": lambda: (W.simple_desc(), W.gen_flat_batch_shuffled(random.Random(42), 65536)),
            # one block alone (64 messages): the block's latency chain with nothing beside it
            "c2one": lambda: (W.simple_desc(), W.gen_flat_batch(random.Random(42), 64))}[cfg]()
n = len(msgs)
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
cnt = (C.c_uint64 * 16)()
args = (ctx.h, dh, flat.root_type, d_json.data_ptr(), d_in.data_ptr(), n, 1, d_out.data_ptr(), d_oo.data_ptr(),
        d_ol.data_ptr(), d_ret.data_ptr())
_lib.check(L.dg_bench_device(*args, 1, C.byref(ms)))
_lib.check(L.dg_ctx_counters(ctx.h, cnt, 16, 1))
reps = 5
_lib.check(L.dg_bench_device(*args, reps, C.byref(ms)))
_lib.check(L.dg_ctx_counters(ctx.h, cnt, 16, 1))
if "--plain" in sys.argv:  # any build: the time only (e.g. under rocprofv3 --pmc)
    print(f"{cfg}: {ms.value / reps * 1000:.1f} us/step")
    sys.exit(0)
if "--stages" in sys.argv:  # a -DDG_FLPROF_G build
    c = list(cnt)[2:8]
    waves = max(1, n // 64 // 32) * 4
    print(f"{cfg}: {ms.value / reps * 1000:.1f} us/step (instrumented)")
    for k, nm in enumerate(["separators", "delimiters", "key", "value", "sizes", "after"]):
        print("  %-12s %8.0f cycles/wave" % (nm, c[k] / reps / waves))
    sys.exit(0)
if fields:
    c = list(cnt)[2:14]
    waves = max(1, n // 64 // 32) * 4
    print(f"{cfg}: {ms.value / reps * 1000:.1f} us/step (instrumented), ok={(d_ret.cpu().numpy() == 0).sum()}")
    for k in range(6):
        print("  field slot %d: parse %8.0f  write %8.0f cycles/wave" % (k, c[k] / reps / waves * 4, c[6 + k] / reps / waves * 4))
    sys.exit(0)
c = list(cnt)[2:10]
names = ["stage+desc+barrier", "classify+scan", "record", "open/close+barrier 1", "parse", "barrier 2", "write+tasks",
         "chunks+barrier 4"]
waves = max(1, n // 64 // 32) * 4  # 4 waves per 64-message block; 1 block in 32 sampled
tot = sum(c)
print(f"{cfg}: {ms.value / reps * 1000:.1f} us/step (instrumented), ok={(d_ret.cpu().numpy() == 0).sum()}")
for k, nm in enumerate(names):
    print("  %-20s %6.2f%%  %9.0f cycles/wave" % (nm, 100 * c[k] / max(1, tot), c[k] / reps / waves))
print("  total %.0f cycles/wave" % (tot / reps / waves))
