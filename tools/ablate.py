"""Time the C2 batch with a given libdgj2t build (DG_LIB_PATH) — ablation runs."""
import os, sys, random, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from dynamicgo_amd import _lib, conv, workloads as W
from dynamicgo_amd.thrift import flatten
import ctypes as C

def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    dev = torch.device("cuda:0")
    if cfg == "c2":
        td, msgs = W.simple_desc(), W.gen_flat_batch(random.Random(42), 65536)
    elif cfg in ("c3small", "c3big"):  # C3 messages that fit the wave kernel's LDS stage, or not
        td, msgs = W.nesting_i64_desc(), W.gen_nested_batch(random.Random(43), 3 * 65536)
        msgs = [m for m in msgs if (len(m) <= 1900) == (cfg == "c3small")][:32768]
        print("%s: %d msgs, %d bytes" % (cfg, len(msgs), sum(map(len, msgs))))
    else:
        td, msgs = W.nesting_i64_desc(), W.gen_nested_batch(random.Random(43), 65536)
    flat = flatten(td)
    a, off = W.arena(msgs)
    n = len(msgs)
    slots = np.zeros(n + 1, dtype=np.int64)
    np.cumsum((np.diff(off).astype(np.int64) * 4 + 64 + 7) // 8 * 8, out=slots[1:])
    ctx = conv.Context(0)
    dh = ctx.desc(flat)
    d_json = torch.from_numpy(a).to(dev); d_in = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_out = torch.empty(int(slots[-1]) + 64, dtype=torch.uint8, device=dev); d_oo = torch.from_numpy(slots).to(dev)
    d_ol = torch.zeros(n, dtype=torch.int32, device=dev); d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
    L = _lib.lib()
    ms = C.c_float(0)
    _lib.check(L.dg_bench_device(ctx.h, dh, flat.root_type, d_json.data_ptr(), d_in.data_ptr(), n, 1, d_out.data_ptr(),
                                 d_oo.data_ptr(), d_ol.data_ptr(), d_ret.data_ptr(), 3, C.byref(ms)))
    _lib.check(L.dg_bench_device(ctx.h, dh, flat.root_type, d_json.data_ptr(), d_in.data_ptr(), n, 1, d_out.data_ptr(),
                                 d_oo.data_ptr(), d_ol.data_ptr(), d_ret.data_ptr(), 20, C.byref(ms)))
    ok = int((d_ret.cpu().numpy() == 0).sum())
    if os.environ.get("DG_PROF"):
        o = d_out.cpu().numpy()
        prof = np.stack([o[int(slots[i]):int(slots[i]) + 128].view(np.uint64) for i in range(0, n, 1)])
        names = ["advance_ns", "read_key", "find_field", "number", "string", "binary", "unset", "TOTAL run",
                 "str.advance", "str.unquote", "str.copy", "str.w32", "bin.b64decode"]
        tot = prof[:, 7].astype(np.float64)
        for k, nm in enumerate(names):
            v = prof[:, k].astype(np.float64)
            print("  %-12s mean %10.0f ticks  (%.1f%% of run)" % (nm, v.mean(), 100 * v.mean() / tot.mean()))
    print("%-40s %s %.1f us/launch  ok=%d" % (os.path.basename(os.environ.get("DG_LIB_PATH", "default")), cfg, ms.value / 20 * 1000, ok))

main()
