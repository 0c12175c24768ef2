"""The benched C4 and C5 batches at their full sizes, byte for byte against the
compiled reference: the same device-resident route bench.py
times (dg_j2t_batch_device_ml, default routing), every message's status word
and Thrift bytes compared with oracle/_ref's j2t_arena, and no message left to
the exact machine. C2 and C3 at full size are in test_gpu_parity.py."""
import random

import numpy as np
import pytest

import oracle
from dynamicgo_amd import _lib, conv, thrift as T, workloads as W

pytestmark = pytest.mark.gpu


def _device_packed(flat, arena, off, flags=1):
    """Convert on the GPU as bench.py does, then pack the used slot prefixes
    back to back (dg_pack_device_scan). Returns (rets, packed bytes, packed
    offsets[n+1], exact-machine messages)."""
    import torch
    dev = torch.device("cuda", 0)
    ctx = conv.default_context()
    L = _lib.lib()
    n = len(off) - 1
    lens = np.diff(off).astype(np.int64)
    slots = np.zeros(n + 1, dtype=np.int64)
    np.cumsum((lens * 4 + 64 + 127) & ~127, out=slots[1:])
    d_json = torch.from_numpy(np.ascontiguousarray(arena)).to(dev)
    d_in = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_out = torch.empty(int(slots[-1]) + 64, dtype=torch.uint8, device=dev)
    d_oo = torch.from_numpy(slots).to(dev)
    d_ol = torch.zeros(n, dtype=torch.int32, device=dev)
    d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
    d_pend = torch.zeros(4, dtype=torch.int32, device=dev)
    ctx.stats(reset=True)
    s = None  # the context's own stream
    _lib.check(L.dg_j2t_batch_device_ml(ctx.h, ctx.desc(flat), flat.root_type, d_json.data_ptr(), d_in.data_ptr(), n,
                                        flags, d_out.data_ptr(), d_oo.data_ptr(), d_ol.data_ptr(), d_ret.data_ptr(),
                                        d_pend.data_ptr(), s, int(lens.max())))
    torch.cuda.synchronize()
    del d_json
    total = int(d_ol.to(torch.int64).sum().item())
    d_dst = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    d_doff = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    _lib.check(L.dg_pack_device_scan(ctx.h, d_out.data_ptr(), d_oo.data_ptr(), d_ol.data_ptr(), n, d_dst.data_ptr(),
                                     d_doff.data_ptr(), s))
    torch.cuda.synchronize()
    bails, _ = ctx.stats(reset=True)
    return (d_ret.cpu().numpy().astype(np.uint64), d_dst[:total].cpu().numpy(), d_doff.cpu().numpy(), bails,
            int(d_pend.sum().item()))


def _reference_packed(flat, arena, off, flags=1):
    """oracle/_ref (the reference's native.c) over the same arena, 8 threads,
    packed the same way."""
    chk = oracle.RefOracle() or oracle.PortOracle()
    rets, (out, oo, ol) = chk.j2t_arena(flat, arena, off, flags, nthreads=8, decode=False)
    n = len(off) - 1
    ok = rets == 0
    assert (ol.astype(np.uint64) <= np.diff(oo))[ok].all(), "reference slot too small"
    lens = np.where(ok, ol, 0).astype(np.int64)
    poff = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=poff[1:])
    packed = np.concatenate([out[int(oo[i]):int(oo[i]) + int(lens[i])] for i in range(n)]) if n else np.zeros(0, np.uint8)
    return rets.astype(np.uint64), packed, poff


def _check_full(flat, arena, off):
    n = len(off) - 1
    g_ret, g_bytes, g_off, bails, pend = _device_packed(flat, arena, off)
    r_ret, r_bytes, r_off = _reference_packed(flat, arena, off)
    assert pend == 0
    bad = np.nonzero(g_ret != r_ret)[0]
    assert bad.size == 0, (bad[:8], [hex(int(g_ret[i])) for i in bad[:8]], [hex(int(r_ret[i])) for i in bad[:8]])
    assert (r_ret == 0).all()
    diff = np.nonzero(g_off != r_off)[0]
    assert diff.size == 0, ("lengths differ from message", int(diff[0]) - 1 if diff.size else None)
    if not np.array_equal(g_bytes, r_bytes):
        at = int(np.nonzero(g_bytes != r_bytes)[0][0])
        i = int(np.searchsorted(r_off, at, side="right")) - 1
        pytest.fail(f"message {i} of {n} differs at byte {at - int(r_off[i])}")
    assert bails == 0, f"{bails} messages went to the exact machine"


def test_full_c4_batch_vs_reference():
    """C4: 4 096 messages of ~85 KB (48 KiB base64 + 1 024 doubles), seed 44,
    the batch bench.py --config c4 converts."""
    fl = T.flatten(W.large_desc())
    msgs = W.gen_large_batch(random.Random(44), 4096)
    a, off = W.arena(msgs)
    del msgs
    _check_full(fl, a, off)


def test_full_c5_batch_vs_reference(c5_batch):
    """C5: ONE 1 048 576-message mixed batch (90 % flat / 9.5 % nested / 0.5 %
    large), seed 45, the batch bench.py --config c5 converts at one rank."""
    a, off = c5_batch
    _check_full(T.flatten(W.mixed_desc()), np.asarray(a), np.asarray(off, dtype=np.uint64))
