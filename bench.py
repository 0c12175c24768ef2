#!/usr/bin/env python3
"""bench.py — conv/j2t device-resident throughput on MI355X.

A "step" = one pass of the hot path (JSON -> Thrift binary, BinaryConv.Do per
message) over one batch that is already resident in HBM. At N GPUs each rank
converts its own batch of the configured workload (weak scaling; messages are
independent, no data-path collective); the flattened descriptor is broadcast
once from rank 0 over RCCL.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5|c1]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line (rank 0). `value` = total JSON bytes converted by all
ranks / max-over-ranks wall time of the K timed steps.
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (first: one HIP runtime per process, see dynamicgo_amd/_lib.py)

from dynamicgo_amd import _lib, workloads as W  # noqa: E402
from dynamicgo_amd.thrift import flatten  # noqa: E402

METRIC = "conv/j2t GB/s JSON in + msgs/s, 64K-batch device-resident, 1→8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PER_MSG_META = 28      # in_off 8 + out_off 8 + out_len 4 + ret 8 bytes

CONFIGS = {
    "c2": ("C2: 65536 flat baseline.Simple messages <=256 B, seed 42", 65536),
    "c3": ("C3: 65536 nested NestingI64 messages (list<string> + map<i64,Simple>), seed 43", 65536),
    "c4": ("C4: 4096 large messages (48 KiB base64 binary + 1024 doubles), seed 44", 4096),
    "c1": ("C1: the reference's Simple payload x 65536 (236 B each)", 65536),
    "c5": ("C5: mixed 90% flat / 9.5% nested / 0.5% large, 131072 per GPU (1M over 8), seed 45", 131072),
}


def make_batch(cfg: str, rank: int):
    if cfg == "c2":
        return W.simple_desc(), W.gen_flat_batch(random.Random(42 + 1000 * rank), CONFIGS[cfg][1])
    if cfg == "c3":
        return W.nesting_i64_desc(), W.gen_nested_batch(random.Random(43 + 1000 * rank), CONFIGS[cfg][1])
    if cfg == "c4":
        return W.large_desc(), W.gen_large_batch(random.Random(44 + 1000 * rank), CONFIGS[cfg][1])
    if cfg == "c1":
        return W.simple_desc(), [W.c1_simple_json()] * CONFIGS[cfg][1]
    if cfg == "c5":
        return W.mixed_desc(), W.gen_mixed_batch(random.Random(45 + 1000 * rank), CONFIGS[cfg][1])
    raise ValueError(cfg)


def cpu_baseline(flat, arena, off, flags, budget_s: float = 12.0):
    """The reference's own native/*.c (oracle/_ref) on this host's cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # reported baseline only
    ref = oracle.RefOracle()
    kind = "reference"
    if ref is None:
        ref, kind = oracle.PortOracle(), "port"
    cores = 1 if kind == "port" else max(1, min(16, (os.cpu_count() or 1)))
    nbytes = int(off[-1] - off[0])
    reps, t_best = 0, None
    t_end = time.perf_counter() + budget_s
    while time.perf_counter() < t_end or reps < 2:
        t0 = time.perf_counter()
        ref.j2t_arena(flat, arena, off, flags, nthreads=cores, decode=False)
        dt = time.perf_counter() - t0
        t_best = dt if t_best is None else min(t_best, dt)
        reps += 1
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(nbytes / t_best / 1e9, 4), "unit": "GB/s", "cores": cores, "kind": kind,
            "sample": f"the full batch ({len(off) - 1} msgs, {nbytes} B) x {reps} reps, best of reps, "
                      f"{cores} threads of '{model}' (nproc={os.cpu_count()})"}


def e2e_host_path(L, ctx, dh, root, flags, arena, off, dev, chunks: int = 8, reps: int = 5):
    """End-to-end from host memory (HTTP bodies in) to host memory (Thrift out):
    pinned H2D of each chunk's JSON + offsets, conversion, device-side packing
    of the outputs (dg_pack_device), D2H of the packed bytes + out_len + ret.
    Chunks alternate between two streams so copies overlap conversion.
    Returns GB/s of JSON in (best of reps) and the serial breakdown."""
    n = len(off) - 1
    bounds = np.linspace(0, n, chunks + 1).astype(np.int64)
    C = []
    for c in range(chunks):
        a, b = int(bounds[c]), int(bounds[c + 1])
        lo, hi = int(off[a]), int(off[b])
        o = (off[a:b + 1] - off[a]).astype(np.int64)
        lens = np.diff(o)
        slots = np.zeros(b - a + 1, dtype=np.int64)
        np.cumsum((lens * 4 + 64 + 7) & ~7, out=slots[1:])
        h_json = torch.from_numpy(np.concatenate([arena[lo:hi], np.zeros(64, np.uint8)])).pin_memory()
        h_in = torch.from_numpy(o).pin_memory()
        C.append(dict(n=b - a, h_json=h_json, h_in=h_in,
                      d_json=torch.empty_like(h_json, device=dev), d_in=torch.empty_like(h_in, device=dev),
                      d_out=torch.empty(int(slots[-1]) + 64, dtype=torch.uint8, device=dev),
                      d_oo=torch.from_numpy(slots).to(dev), d_ol=torch.zeros(b - a, dtype=torch.int32, device=dev),
                      d_ret=torch.zeros(b - a, dtype=torch.int64, device=dev),
                      d_doff=torch.zeros(b - a + 1, dtype=torch.int64, device=dev),
                      d_pack=torch.empty(int(slots[-1]) + 64, dtype=torch.uint8, device=dev),
                      h_ol=torch.empty(b - a, dtype=torch.int32).pin_memory(),
                      h_ret=torch.empty(b - a, dtype=torch.int64).pin_memory()))
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]

    def run(sizes):
        for k, c in enumerate(C):
            st = streams[k % 2]
            with torch.cuda.stream(st):
                c["d_json"].copy_(c["h_json"], non_blocking=True)
                c["d_in"].copy_(c["h_in"], non_blocking=True)
                _lib.check(L.dg_j2t_batch_device(ctx.h, dh, root, c["d_json"].data_ptr(), c["d_in"].data_ptr(), c["n"],
                                                 flags, c["d_out"].data_ptr(), c["d_oo"].data_ptr(), c["d_ol"].data_ptr(),
                                                 c["d_ret"].data_ptr(), None, st.cuda_stream))
                torch.cumsum(c["d_ol"], 0, dtype=torch.int64, out=c["d_doff"][1:])
                _lib.check(L.dg_pack_device(ctx.h, c["d_out"].data_ptr(), c["d_oo"].data_ptr(), c["d_ol"].data_ptr(),
                                            c["n"], c["d_pack"].data_ptr(), c["d_doff"].data_ptr(), st.cuda_stream))
                c["h_ol"].copy_(c["d_ol"], non_blocking=True)
                c["h_ret"].copy_(c["d_ret"], non_blocking=True)
                if sizes is not None:
                    c["h_pack"][:sizes[k]].copy_(c["d_pack"][:sizes[k]], non_blocking=True)
        for st in streams:
            st.synchronize()

    run(None)  # warm-up: learn each chunk's packed size (deterministic)
    sizes = [int(c["h_ol"].to(torch.int64).sum()) for c in C]
    for c, sz in zip(C, sizes):
        c["h_pack"] = torch.empty(max(sz, 1), dtype=torch.uint8).pin_memory()
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(sizes)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    # what came back is what the kernel wrote: packed bytes == the slots' used prefixes
    c = C[0]
    slots_h, oo_h, ol_h = c["d_out"].cpu().numpy(), c["d_oo"].cpu().numpy(), c["h_ol"].numpy()
    want = b"".join(slots_h[int(oo_h[i]):int(oo_h[i]) + int(ol_h[i])].tobytes() for i in range(c["n"]))
    if c["h_pack"][:sizes[0]].numpy().tobytes() != want[:sizes[0]]:
        raise RuntimeError("e2e: packed output differs from the device slots")
    json_bytes = int(off[-1] - off[0])
    return {"value": round(json_bytes / best / 1e9, 3), "unit": "GB/s", "ms": round(best * 1e3, 3),
            "thrift_bytes": sum(sizes), "chunks": chunks, "streams": 2,
            "method": "pinned H2D (JSON+offsets) -> convert -> dg_pack_device -> D2H (packed Thrift + out_len + ret), "
                      "chunks alternating over 2 streams, wall clock, best of %d" % reps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory end-to-end measurement")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.distributed.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    from dynamicgo_amd import conv
    td, msgs = make_batch(args.config, rank)
    flat = flatten(td)
    flags = 1  # conv.Options{} -> F_ALLOW_UNKNOWN (conv/j2t/conv.go:102-104)

    # descriptor: built on rank 0, broadcast over RCCL, created from device memory
    L = _lib.lib()
    ctx = conv.Context(local)
    if dist:
        from dynamicgo_amd import dist as D
        import ctypes as C
        blob = D.broadcast_blob(flat.blob if rank == 0 else None, dev)  # RCCL over xGMI
        h = C.c_void_p()
        _lib.check(L.dg_desc_create_device(ctx.h, blob.data_ptr(), blob.numel(), C.byref(h)))
        ctx._descs[flat.blob] = h
    dh = ctx.desc(flat)

    arena, off = W.arena(msgs)
    n = len(msgs)
    lens = np.diff(off).astype(np.int64)
    max_len = int(lens.max())  # known to the host that built the arena (dg_j2t_batch_device_ml)
    slots = np.zeros(n + 1, dtype=np.int64)
    np.cumsum((lens * 4 + 64 + 7) & ~7, out=slots[1:])  # dg_slot_bound: 8-aligned slots
    d_json = torch.from_numpy(arena).to(dev)
    d_in = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_out = torch.empty(int(slots[-1]) + 64, dtype=torch.uint8, device=dev)
    d_oo = torch.from_numpy(slots).to(dev)
    d_ol = torch.zeros(n, dtype=torch.int32, device=dev)
    d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
    d_pend = torch.zeros(4, dtype=torch.int32, device=dev)
    # a real (non-null) stream: the kernels and the timing events share it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)

    def step():
        _lib.check(L.dg_j2t_batch_device_ml(ctx.h, dh, flat.root_type, d_json.data_ptr(), d_in.data_ptr(), n, flags,
                                         d_out.data_ptr(), d_oo.data_ptr(), d_ol.data_ptr(), d_ret.data_ptr(),
                                         d_pend.data_ptr(), stream.cuda_stream, max_len))

    ctx.stats(reset=True)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    bails, deeps = ctx.stats(reset=True)
    # correctness of what we time: every message converted, none left pending
    rets = d_ret.cpu().numpy()
    ok = int((rets == 0).sum())
    if int(d_pend.sum().item()) != 0 or ok != n:
        print(f"[rank {rank}] WARNING: {n - ok} messages not ok", file=sys.stderr)
    json_bytes = int(off[-1])
    thrift_bytes = int(d_ol.to(torch.int64).sum().item())
    alg_bytes = json_bytes + thrift_bytes + PER_MSG_META * n

    # timed region
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    wall = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1) / args.steps  # HIP events on the launch stream
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if dist:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    wall_max = float(t.item())

    total_json = json_bytes * world
    value = total_json / wall_max * args.steps / 1e9
    msgs_per_s = n * world * args.steps / wall_max
    achieved = alg_bytes / (gpu_ms / 1e3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(flat, arena, off, flags)
    e2e = None
    if rank == 0 and not args.no_e2e:
        e2e = e2e_host_path(L, ctx, dh, flat.root_type, flags, arena, off, dev)

    traffic = None
    tp = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tp):
        with open(tp) as fh:
            traffic = json.load(fh).get("hbm_bytes_per_launch")

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(wall_max / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": CONFIGS[args.config][0], "global_batch": n * world, "msgs_per_rank": n,
                       "avg_json_bytes": round(json_bytes / n, 1), "msgs_per_s": round(msgs_per_s),
                       "thrift_bytes_per_rank": thrift_bytes, "flags": flags,
                       "parallelism": f"dp{world} (independent shards, descriptor RCCL-broadcast)",
                       "ok_msgs_per_rank": ok,
                       "exact_path_msgs_per_step": bails / max(1, args.warmup),
                       "deep_msgs_per_step": deeps / max(1, args.warmup)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "kernel_ms": round(gpu_ms, 5), "alg_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
            "e2e_host": e2e,
        }
        print(json.dumps(line), flush=True)
    if dist:
        torch.distributed.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
