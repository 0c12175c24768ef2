#!/usr/bin/env python3
"""bench.py — conv/j2t device-resident throughput on MI355X.

A "step" = one pass of the hot path (JSON -> Thrift binary, BinaryConv.Do per
message) over one batch that is already resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c2x|c2s|c3|c4|c5|c1|t2j-c2|t2j-c3]

Multi-GPU: with --gpus N > 1 and no WORLD_SIZE in the environment this
process launches N ranks itself (one process per GPU, RANK/LOCAL_RANK/
WORLD_SIZE/MASTER_ADDR=127.0.0.1/MASTER_PORT set, before anything touches
the GPU) and exits with their status; under torchrun it is one of the ranks.
Messages are independent, so no data-path collective exists: the flattened
descriptor is broadcast once from rank 0 (RCCL over xGMI) and every rank
converts its own shard.
  * c2/c2x/c2s/c3/c4/c1 — weak scaling: every rank converts a batch of the
    config's size (rank r draws with seed + 1000 r), global batch = N x size.
  * c5 — strong scaling: ONE 1 048 576-message mixed batch (seed 45), split
    into N byte-balanced contiguous shards (dist.shard_ranges), rank r
    converts shard r.
Prints ONE JSON line (rank 0). `value` = JSON bytes converted by all ranks /
max-over-ranks wall time of the K timed steps (barrier + synchronize on both
sides).
"""
import argparse
import json
import os
import random
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "conv/j2t GB/s JSON in + msgs/s, 64K-batch device-resident, 1→8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PER_MSG_META = 28      # in_off 8 + out_off 8 + out_len 4 + ret 8 bytes
CPU_SHARE = 16         # host CPUs the GPU box grants per GPU

CONFIGS = {
    "c2": ("C2: 65536 flat baseline.Simple messages <=256 B, seed 42", 65536, "weak"),
    "c2x": ("C2 with the reference benchmark's options (WriteDefaultField + EnableValueMapping, flags 0x7; "
            "testdata/test/baseline_j2t_test.go:721-737): 65536 flat Simple messages, seed 42", 65536, "weak"),
    "c2s": ("C2 divergence stress: 65536 flat Simple messages with the keys of every message in a random "
            "order, seed 42", 65536, "weak"),
    "c3": ("C3: 65536 nested NestingI64 messages (list<string> + map<i64,Simple>), seed 43", 65536, "weak"),
    "c4": ("C4: 4096 large messages (48 KiB base64 binary + 1024 doubles), seed 44", 4096, "weak"),
    "c1": ("C1: the reference's Simple payload (236 B) x 65536", 65536, "weak"),
    "c5": ("C5: ONE 1048576-message mixed batch (90% flat / 9.5% nested / 0.5% large), seed 45, "
           "byte-balanced shards over the ranks", 1 << 20, "strong"),
    # the reverse path (conv/t2j): the Thrift bytes of a j2t
    # config (converted on the GPU at setup, packed in HBM) back to JSON
    "t2j-c2": ("t2j over C2: the Thrift of 65536 flat Simple messages (seed 42) -> JSON", 65536, "weak"),
    "t2j-c3": ("t2j over C3: the Thrift of 65536 nested NestingI64 messages (seed 43) -> JSON", 65536, "weak"),
    # the drop-in path: BinaryConv.Do called once per
    # message from many threads, coalesced by the batching aggregator
    "agg": ("BinaryConv.Do per message from 16 OS threads (up to 8192 calls in flight each) through the batching "
            "aggregator dg_agg: the 65536 C2 messages (seed 42) x 4 = 262144 calls per step, host memory in and out",
            262144, "weak"),
}
AGG_METRIC = "conv/j2t BinaryConv.Do calls/s through the batching aggregator (host memory in/out), 16 threads"
T2J_METRIC = "conv/t2j GB/s Thrift in + msgs/s, 64K-batch device-resident"
# batches in flight in the timed steps (default 2). Measured one at a time
# faster or equal: C5's 1M batch (4.45 vs 4.73 ms), t2j-c3 (1.48 vs 1.50 ms;
# its wave kernel's workspace is ordered across streams)
DEFAULT_INFLIGHT = {"c5": 1, "t2j-c3": 1}
KERNEL_NAMES = (("j2t_flat_kernel", "j2t_small_kernel"), "j2t_wave_kernel")  # first launch (flat | small), wave
FLAGS = {"c2x": 0x7}  # default: conv.Options{} -> F_ALLOW_UNKNOWN (conv/j2t/conv.go:102-104)


# ---------------------------------------------------------------- launching
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv, python=sys.executable, script=None) -> int:
    """One child process per GPU running this script with the same args, the
    torch.distributed env set; returns the worst exit status. The parent
    never touches the GPU (children are started, not exec'd)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([python, script or os.path.abspath(__file__), *argv], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


# ---------------------------------------------------------------- workloads
def rank_workload(cfg: str, rank: int, world: int, workers: int = 1, c5_n: int = None, c5_scale: float = 1.0):
    """This rank's (TypeDescriptor, arena, offsets, meta). Weak configs: a
    batch of the config's size per rank; c5: shard `rank` of the one global
    batch (byte-balanced contiguous ranges, dist.shard_ranges)."""
    from dynamicgo_amd import workloads as W
    from dynamicgo_amd.dist import shard_ranges
    size = CONFIGS[cfg][1]
    if cfg == "c5":
        n = c5_n or size
        # generated once per node (/dev/shm), mapped by every rank; DG_C5_CACHE=1
        # also at one rank (a profiler run: no generator pool under the tool)
        if world > 1 or os.environ.get("DG_C5_CACHE"):
            a, off = c5_shared_arena(n, 45, c5_scale, gen_workers())
        else:
            a, off = W.gen_mixed_arena(n, 45, workers=workers, large_scale=c5_scale)
        lo, hi = shard_ranges(off, world)[rank]
        sa, so = W.arena_slice(a, off, lo, hi)
        del a
        return W.mixed_desc(), sa, so, {"global_batch": n, "global_json_bytes": int(off[-1]), "shard": [lo, hi]}
    if cfg.startswith("t2j-"):
        cfg = cfg[4:]
    if cfg == "agg":
        rng = random.Random(42 + 1000 * rank)
        msgs = W.gen_flat_batch(rng, 65536)
        a, off = W.arena(msgs * (size // 65536))
        return W.simple_desc(), a, off, {"global_batch": size * world, "global_json_bytes": None, "shard": None,
                                         "unique": 65536}
    rng = random.Random({"c2": 42, "c2x": 42, "c2s": 42, "c3": 43, "c4": 44, "c1": 0}[cfg] + 1000 * rank)
    if cfg in ("c2", "c2x"):
        td, msgs = W.simple_desc(), W.gen_flat_batch(rng, size)
    elif cfg == "c2s":
        td, msgs = W.simple_desc(), W.gen_flat_batch_shuffled(rng, size)
    elif cfg == "c3":
        td, msgs = W.nesting_i64_desc(), W.gen_nested_batch(rng, size)
    elif cfg == "c4":
        td, msgs = W.large_desc(), W.gen_large_batch(rng, size)
    else:
        td, msgs = W.simple_desc(), [W.c1_simple_json()] * size
    a, off = W.arena(msgs)
    return td, a, off, {"global_batch": size * world, "global_json_bytes": None, "shard": None}


def gen_workers() -> int:
    """Worker processes for generating the C5 batch: the CPUs this process may
    use (the ranks of one node wait for the one that generates)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(2, min(n, 32))


def _c5_cache_base(n: int, seed: int, scale: float) -> str:
    job = os.environ.get("MASTER_PORT", "0")
    return f"/dev/shm/dgj2t_c5_{n}_{seed}_{scale}_{job}"


def c5_shared_arena(n: int, seed: int, scale: float, workers: int):
    """The ONE C5 batch of a multi-rank run: the first rank to take the lock
    generates it (all its CPUs) into /dev/shm; the others wait for the lock and
    map the same files read-only. release_c5_cache() unlinks them once every
    rank has sliced its shard."""
    import fcntl
    from dynamicgo_amd import workloads as W
    base = _c5_cache_base(n, seed, scale)
    with open(base + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not (os.path.exists(base + ".off.npy") and os.path.exists(base + ".arena.npy")):
            a, off = W.gen_mixed_arena(n, seed, workers=workers, large_scale=scale)
            for name, arr in (("arena", a), ("off", off)):
                tmp = f"{base}.{name}.tmp.npy"
                np.save(tmp, arr)
                os.replace(tmp, f"{base}.{name}.npy")
            del a, off
        fcntl.flock(lk, fcntl.LOCK_UN)
    return np.load(base + ".arena.npy", mmap_mode="r"), np.load(base + ".off.npy")


def release_c5_cache(n: int = None, seed: int = 45, scale: float = 1.0):
    """Unlink the node's C5 cache (call after a barrier: every rank has its shard)."""
    base = _c5_cache_base(n or CONFIGS["c5"][1], seed, scale)
    for suf in (".arena.npy", ".off.npy", ".lock"):
        try:
            os.unlink(base + suf)
        except FileNotFoundError:
            pass


def share_descriptor(flat, rank: int, dev, backend: str):
    """Rank 0's flattened descriptor on every rank, as a uint8 tensor on `dev`
    (RCCL broadcast straight into device memory; gloo via host memory)."""
    import torch
    from dynamicgo_amd import dist as D
    where = dev if backend == "nccl" else torch.device("cpu")
    t = D.broadcast_blob(flat.blob if rank == 0 else None, where)
    return t.to(dev) if t.device != dev else t


# ---------------------------------------------------------------- CPU baseline
def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _read(path: str):
    try:
        with open(path) as fh:
            return fh.read().strip()
    except OSError:
        return None


def host_cpu_env() -> dict:
    """What bounds the CPU baseline on this host: the affinity mask, the
    cgroup CPU quota (v2 cpu.max, or v1 cfs quota/period) and throttling
    counters, and the load average. A quota below the threads the baseline
    runs (e.g. 16 CPUs of quota under a 128-CPU affinity) throttles them in
    every quota period: the all-core passes then swing by large factors."""
    env = {"affinity_cpus": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(),
           "loadavg": [round(x, 2) for x in os.getloadavg()]}
    v2 = _read("/sys/fs/cgroup/cpu.max")
    if v2:
        q, per = (v2.split() + ["100000"])[:2]
        env["cgroup_cpu_max"] = v2
        env["quota_cpus"] = None if q == "max" else round(int(q) / int(per), 2)
    else:
        q, per = _read("/sys/fs/cgroup/cpu/cpu.cfs_quota_us"), _read("/sys/fs/cgroup/cpu/cpu.cfs_period_us")
        if q and per:
            env["cgroup_cfs"] = f"{q} {per}"
            env["quota_cpus"] = None if int(q) < 0 else round(int(q) / int(per), 2)
    st = _read("/sys/fs/cgroup/cpu.stat") or _read("/sys/fs/cgroup/cpu/cpu.stat")
    if st:
        kv = dict(line.split()[:2] for line in st.splitlines() if len(line.split()) >= 2)
        env["throttle"] = {k: int(kv[k]) for k in ("nr_periods", "nr_throttled", "throttled_usec", "throttled_time")
                           if k in kv}
    return env


def cpu_baseline(flat, arena, off, flags, budget_s: float = 6.0):
    """The reference's own native/*.c (oracle/_ref, clang -O3 like the
    reference's build) on this host, outputs preallocated and first touched by
    an untimed pass, median of reps, byte-balanced shards, threads pinned to
    distinct physical cores:
      * value: the cores that can actually run at once, i.e. the physical
        cores of the affinity mask capped by the cgroup CPU quota (16 on the
        GPU box: more threads than the quota only throttle);
      * all_affinity: one thread per physical core of the affinity mask
        (SURVEY.md §8(d)), reported beside it with the quota's throttling;
      * one core over a bounded prefix."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # reported baseline only
    ref = oracle.RefOracle()
    if ref is None:
        return None
    phys, logical = oracle.physical_cpus()
    cores_all = max(1, len(phys))
    quota = host_cpu_env().get("quota_cpus")
    cores = max(1, min(CPU_SHARE, len(phys), int(quota) if quota else len(phys)))
    n = len(off) - 1
    nbytes = int(off[-1] - off[0])

    def timed(a, o, cpus, per=1):
        t1 = ref.j2t_timed(flat, a, o, flags, cpus, 1)
        reps = int(max(5, min(200, budget_s / 2 / max(t1, 1e-6))))
        ts = []
        ref.j2t_timed(flat, a, o, flags, cpus, reps, times=ts)
        ts = [t / per for t in ts]
        return float(np.median(ts)), ts

    # a pass of a small batch takes ~1 ms on 16 cores, where one descheduled
    # thread doubles it (r7z C2: passes spread 4x); the timed passes convert
    # the batch `rep` times over (the same messages, a >= 64 MB arena), and
    # the times are per batch
    rep = int(max(1, min(16, (64 << 20) // max(nbytes, 1))))
    if rep > 1:
        body = np.asarray(arena[int(off[0]):int(off[-1])])
        arena_r = np.concatenate([body] * rep + [np.zeros(64, dtype=np.uint8)])
        off_r = np.concatenate([(off[:n] - off[0]) + k * nbytes for k in range(rep)] +
                               [np.array([rep * nbytes], dtype=off.dtype)]).astype(np.uint64)
    else:
        arena_r, off_r = arena, off
    env_s = host_cpu_env()
    t_share, ts_share = timed(arena_r, off_r, phys[:cores], rep)
    env0 = host_cpu_env()
    t_all, ts_all = (t_share, ts_share) if cores == cores_all else timed(arena_r, off_r, phys[:cores_all], rep)
    env1 = host_cpu_env()
    # one core: a prefix of at most ~64 MB / 65536 messages
    k = int(min(n, 65536, max(1, np.searchsorted(off, off[0] + 64 * 1024 * 1024))))
    a1, o1 = arena[:int(off[k]) + 64], off[:k + 1]
    t_one, ts_one = timed(a1, o1, phys[:1])
    one_bytes = int(o1[-1] - o1[0])
    spread = lambda nb, ts: {"min": round(nb / max(ts) / 1e9, 4), "max": round(nb / min(ts) / 1e9, 4),
                             "p5": round(nb / float(np.percentile(ts, 95)) / 1e9, 4),
                             "p95": round(nb / float(np.percentile(ts, 5)) / 1e9, 4),
                             "best_of_5": round(nb / min(ts[:5]) / 1e9, 4)}
    def throttled(a, b):
        if "throttle" in a and "throttle" in b:
            return {k: b["throttle"][k] - a["throttle"].get(k, 0) for k in b["throttle"]}
        return None

    v_share = nbytes / t_share / 1e9
    return {"value": round(v_share, 4), "unit": "GB/s", "cores": cores, "kind": "reference",
            "stat": "median of the passes", "range": spread(nbytes, ts_share),
            "range_ratio": round(max(ts_share) / min(ts_share), 3),
            "range_ratio_p5_p95": round(float(np.percentile(ts_share, 95) / np.percentile(ts_share, 5)), 3),
            "cpu_model": cpu_model(), "msgs_per_s": round(n / t_share),
            "per_core_gbs": round(v_share / cores, 4), "throttling_delta": throttled(env_s, env0),
            "cores_rule": f"min({CPU_SHARE} CPUs per GPU, physical cores in affinity {len(phys)}, "
                          f"cgroup quota {quota})",
            "all_affinity": {"cores": cores_all, "value": round(nbytes / t_all / 1e9, 4),
                             "msgs_per_s": round(n / t_all), "range": spread(nbytes, ts_all),
                             "throttling_delta": throttled(env0, env1),
                             "note": "one thread per physical core of the affinity mask; above the quota the "
                                     "threads only share the quota's CPU time"},
            "one_core_gbs": round(one_bytes / t_one / 1e9, 4), "one_core_ns_per_msg": round(t_one / k * 1e9, 1),
            "one_core_range": spread(one_bytes, ts_one),
            "host": env_s,
            "sample": f"the rank's whole batch ({n} msgs, {nbytes} B; {rep} copies per timed pass, times per "
                      f"batch), median (min/max in range) of "
                      f"{len(ts_share)} passes, {cores} threads pinned to distinct physical cores of "
                      f"'{cpu_model()}' (affinity: {logical} logical CPUs = {len(phys)} physical cores, quota "
                      f"{quota} CPUs); all_affinity: {cores_all} threads, {len(ts_all)} passes; one-core: first "
                      f"{k} msgs ({one_bytes} B), {len(ts_one)} passes; reference native.c built by "
                      f"oracle/Makefile (clang -O3 -mavx2)"}


# ---------------------------------------------------------------- end to end
E2E_CHUNKS = (1, 2, 4, 8, 16)


def e2e_host_path(L, ctx, dh, root, flags, arena, off, dev, flat, reps: int = 5):
    """End-to-end from host memory (HTTP bodies in) to host memory (Thrift
    out) through dg_j2t_pipeline_host: the batch is streamed in `chunks`
    pieces over 3 streams, each piece one pinned H2D of its offsets + JSON,
    conversion, device packing, and a download of [ret | packed offsets]
    then exactly the packed bytes, all issued from C (no per-chunk Python).
    Host buffers are pinned. Every chunking's output is checked against the
    oracle once, outside the timed loop. Returns GB/s of JSON in for the
    best chunking (best of reps each) and the link rates measured alone."""
    import torch
    import ctypes as C
    from dynamicgo_amd import _lib
    n = len(off) - 1
    json_bytes = int(off[-1] - off[0])
    h_json = torch.from_numpy(np.ascontiguousarray(arena[:json_bytes + 64])).pin_memory()
    h_in = torch.from_numpy(off.astype(np.int64)).pin_memory()
    cap = json_bytes * 4 + 80 * n + 64
    h_out = torch.empty(cap, dtype=torch.uint8).pin_memory()
    h_oo = torch.zeros(n + 1, dtype=torch.int64).pin_memory()
    h_ret = torch.zeros(max(n, 1), dtype=torch.int64).pin_memory()
    need = C.c_uint64(0)

    def run(chunks):
        _lib.check(L.dg_j2t_pipeline_host(ctx.h, dh, root, h_json.data_ptr(), h_in.data_ptr(), n, flags, chunks,
                                          h_out.data_ptr(), cap, h_oo.data_ptr(), h_ret.data_ptr(), C.byref(need)))

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # checker only, outside the timed loop
    chk = oracle.RefOracle() or oracle.PortOracle()
    er, eo = chk.j2t_arena(flat, arena, off, flags, nthreads=min(CPU_SHARE, os.cpu_count() or 1))
    sweep = {}
    for chunks in E2E_CHUNKS:
        run(chunks)  # warm: buffers sized, and the result checked
        ob, oo, rr = h_out.numpy(), h_oo.numpy(), h_ret.numpy()
        bad = sum(1 for i in range(n) if int(rr[i]) != int(er[i]) or ob[oo[i]:oo[i + 1]].tobytes() != eo[i])
        if bad:
            raise RuntimeError(f"e2e: {bad} messages differ from the oracle (chunks={chunks})")
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            run(chunks)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        sweep[chunks] = best
    kbest = min(sweep, key=sweep.get)
    thrift = int(h_oo[-1])
    # the copies alone, same sizes (what the link sustains here)
    d_all = torch.empty(json_bytes, dtype=torch.uint8, device=dev)
    d_back = torch.empty(max(thrift, 1), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d_all.copy_(h_json[:json_bytes], non_blocking=True)
    torch.cuda.synchronize()
    t_h2d = time.perf_counter() - t0
    t0 = time.perf_counter()
    h_out[:max(thrift, 1)].copy_(d_back, non_blocking=True)
    torch.cuda.synchronize()
    t_d2h = time.perf_counter() - t0
    return {"value": round(json_bytes / sweep[kbest] / 1e9, 3), "unit": "GB/s", "ms": round(sweep[kbest] * 1e3, 3),
            "chunks": kbest, "sweep_gbs": {str(k): round(json_bytes / v / 1e9, 3) for k, v in sweep.items()},
            "thrift_bytes": thrift, "checked_vs_oracle": n * len(E2E_CHUNKS),
            "h2d_gbs_alone": round(json_bytes / t_h2d / 1e9, 2), "d2h_gbs_alone": round(thrift / t_d2h / 1e9, 2),
            "serial_copy_bound_gbs": round(json_bytes / (t_h2d + t_d2h) / 1e9, 2),
            "method": "dg_j2t_pipeline_host (pinned host buffers): per chunk H2D offsets + JSON -> convert -> pack "
                      "-> D2H ret + packed offsets, then the packed bytes; 3 streams, issued from C; wall clock, "
                      "best of %d per chunking" % reps}


def same_outputs(d_oo, d_ol, a, b) -> bool:
    """Whether two output buffers with the same slots (d_oo, int64 n+1) hold
    the same bytes in every message's slot prefix of d_ol bytes (the slot
    tails are never written)."""
    import torch
    n = d_ol.numel()
    if n == 0 or int(d_oo[-1].item()) == 0:
        return True
    step = 1 << 16  # messages per pass: the masks stay a few hundred MB at C5's slot sizes
    for i in range(0, n, step):
        j = min(n, i + step)
        lo, hi = int(d_oo[i].item()), int(d_oo[j].item())
        oo = d_oo[i:j + 1] - lo
        seg = torch.repeat_interleave(torch.arange(j - i, device=d_oo.device), oo[1:] - oo[:-1])
        pos = torch.arange(hi - lo, device=d_oo.device) - oo[:-1][seg]
        valid = pos < d_ol[i:j].to(torch.int64)[seg]
        del seg, pos
        if not torch.equal(a[lo:hi][valid], b[lo:hi][valid]):
            return False
    return True


# ---------------------------------------------------------------- t2j
def cpu_baseline_t2j(flat, side, arena, off, opts, budget_s: float = 8.0):
    """The t2j checker (oracle/ref_harness.c dgref_t2j: conv/t2j's control
    flow restated in C over the reference's own native encoders) on this
    host, pinned like cpu_baseline: a port, not the Go reference itself."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # reported baseline only
    ref = oracle.RefT2JOracle()
    if ref is None:
        return None
    phys, logical = oracle.physical_cpus()
    cores = max(1, min(CPU_SHARE, len(phys)))
    n = len(off) - 1
    nbytes = int(off[-1] - off[0])
    t1 = ref.t2j_timed(flat, side, arena, off, opts, phys[:cores], 1)
    reps = int(max(5, min(200, budget_s / 2 / max(t1, 1e-6))))
    ts, ts1 = [], []
    ref.t2j_timed(flat, side, arena, off, opts, phys[:cores], reps, times=ts)
    ref.t2j_timed(flat, side, arena, off, opts, phys[:1], 3, times=ts1)
    t_all, t_one = float(np.median(ts)), float(np.median(ts1))
    return {"value": round(nbytes / t_all / 1e9, 4), "unit": "GB/s", "cores": cores, "kind": "port",
            "stat": "median of the passes",
            "range": {"min": round(nbytes / max(ts) / 1e9, 4), "max": round(nbytes / min(ts) / 1e9, 4)},
            "msgs_per_s": round(n / t_all), "one_core_gbs": round(nbytes / t_one / 1e9, 4),
            "sample": f"the rank's whole Thrift batch ({n} msgs, {nbytes} B), median (min/max in range) of {reps} "
                      f"passes, {cores} threads pinned to distinct physical cores of '{cpu_model()}' ({logical} "
                      f"logical CPUs allowed); one-core: same batch, median of 3; oracle/ref_harness.c "
                      f"dgref_t2j_timed (conv/t2j restated in C over the reference's native "
                      f"quote/i64toa/f64toa/b64encode, clang -O3)"}


def bench_t2j(args, rank, world, dev, dist, backend, td, arena, off, meta):
    """t2j configs: the j2t config's batch is converted to Thrift once on the
    GPU (setup, untimed) and packed back to back in HBM; a step converts that
    whole Thrift batch to JSON (dg_t2j_batch_device)."""
    import torch
    import ctypes as C
    from dynamicgo_amd import _lib, conv
    from dynamicgo_amd.thrift import flatten, flatten_t2j
    flat = flatten(td)
    side = flatten_t2j(flat)
    L = _lib.lib()
    ctx = conv.Context(dev.index)
    dh = ctx.desc_t2j(flat)
    n = len(off) - 1
    lens = np.diff(off).astype(np.int64)
    slots = np.zeros(n + 1, dtype=np.int64)
    np.cumsum((lens * 4 + 64 + 127) & ~127, out=slots[1:])  # dg_slot_bound
    d_json = torch.from_numpy(arena).to(dev)
    d_in = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_j2t = torch.empty(int(slots[-1]) + 64, dtype=torch.uint8, device=dev)
    d_oo = torch.from_numpy(slots).to(dev)
    d_ol = torch.zeros(n, dtype=torch.int32, device=dev)
    d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
    d_thrift = torch.zeros(int(slots[-1]) + 64, dtype=torch.uint8, device=dev)
    d_toff = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    _lib.check(L.dg_j2t_batch_device(ctx.h, dh, flat.root_type, d_json.data_ptr(), d_in.data_ptr(), n, 1,
                                     d_j2t.data_ptr(), d_oo.data_ptr(), d_ol.data_ptr(), d_ret.data_ptr(), None,
                                     stream.cuda_stream))
    _lib.check(L.dg_pack_device_scan(ctx.h, d_j2t.data_ptr(), d_oo.data_ptr(), d_ol.data_ptr(), n,
                                     d_thrift.data_ptr(), d_toff.data_ptr(), stream.cuda_stream))
    torch.cuda.synchronize()
    if int((d_ret != 0).sum().item()):
        raise RuntimeError("t2j bench: the j2t setup pass failed on some messages")
    toff = d_toff.cpu().numpy().astype(np.uint64)
    thrift_bytes = int(toff[-1])
    h_thrift = d_thrift[:thrift_bytes + 64].cpu().numpy()
    tl = np.diff(toff).astype(np.int64)
    jslots = np.zeros(n + 1, dtype=np.int64)
    np.cumsum((tl * 3 + 64 + 127) & ~127, out=jslots[1:])  # dg_t2j_slot_bound: 128-byte slots
    t_max = int(tl.max()) if n else 0  # the longest Thrift message: picks the kernel's lanes per message
    del d_j2t, d_json
    d_out = torch.empty(int(jslots[-1]) + 64, dtype=torch.uint8, device=dev)
    d_jo = torch.from_numpy(jslots).to(dev)
    d_jl = torch.zeros(n, dtype=torch.int32, device=dev)
    d_jr = torch.zeros(n, dtype=torch.int64, device=dev)
    opts = 0

    def step():
        _lib.check(L.dg_t2j_batch_device_ml(ctx.h, dh, flat.root_type, d_thrift.data_ptr(), d_toff.data_ptr(), n,
                                            opts, d_out.data_ptr(), d_jo.data_ptr(), d_jl.data_ptr(),
                                            d_jr.data_ptr(), stream.cuda_stream, t_max))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    rets = d_jr.cpu().numpy()
    ok = int((rets == 0).sum())
    if ok != n:
        print(f"[rank {rank}] WARNING: {n - ok} t2j messages not ok", file=sys.stderr)
    json_out = int(d_jl.to(torch.int64).sum().item())
    # parity spot check (outside the timed region): the first 2048 messages
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # checker only
    chk = oracle.RefT2JOracle()
    checked = 0
    if chk is not None and rank == 0:
        out_h, jl_h = d_out.cpu().numpy(), d_jl.cpu().numpy()
        for i in range(min(n, 2048)):
            m = h_thrift[int(toff[i]):int(toff[i + 1])].tobytes()
            er, eo = chk.t2j(flat, side, m, opts)
            got = out_h[int(jslots[i]):int(jslots[i]) + int(jl_h[i])].tobytes()
            if er != int(rets[i]) or eo != got:
                raise RuntimeError(f"t2j bench: message {i} differs from the checker")
            checked += 1
    alg_bytes = thrift_bytes + json_out + PER_MSG_META * n
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # serial leg (one batch at a time): the per-launch time the roofline is priced on
    torch.cuda.synchronize()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    gpu_ms = ev0.elapsed_time(ev1) / args.steps
    # timed steps: `depth` batches in flight, batch k on stream k % depth into
    # output set k % depth (forked from / joined into the launch stream); the
    # library keeps per-stream scratch and orders its shared workspaces by events
    depth = max(1, min(8, args.inflight if args.inflight is not None else DEFAULT_INFLIGHT.get(args.config, 2)))
    sets = [(stream, d_out, d_jl, d_jr)] + [(torch.cuda.Stream(dev), torch.empty_like(d_out), torch.zeros_like(d_jl),
                                              torch.zeros_like(d_jr)) for _ in range(depth - 1)]

    def step_inflight(k):
        for j in range(1, depth):
            sets[j][0].wait_stream(stream)
        for i in range(k):
            st, o, jl, jr = sets[i % depth]
            _lib.check(L.dg_t2j_batch_device_ml(ctx.h, dh, flat.root_type, d_thrift.data_ptr(), d_toff.data_ptr(), n,
                                                opts, o.data_ptr(), d_jo.data_ptr(), jl.data_ptr(), jr.data_ptr(),
                                                st.cuda_stream, t_max))
        for j in range(1, depth):
            stream.wait_stream(sets[j][0])

    if depth > 1:  # warm the streams; every set converts the batch like the serial leg
        step_inflight(args.warmup * depth)
        torch.cuda.synchronize()
        for _, o, jl, jr in sets[1:]:
            if not (torch.equal(jr, d_jr) and torch.equal(jl, d_jl) and same_outputs(d_jo, d_jl, o, d_out)):
                raise SystemExit("t2j in-flight output set differs from the serial one")
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    step_inflight(args.steps)
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    wall = time.perf_counter() - t0
    stats = torch.tensor([wall, float(thrift_bytes), float(n), gpu_ms], dtype=torch.float64,
                         device=dev if backend == "nccl" else "cpu")
    if dist:
        gathered = [torch.zeros_like(stats) for _ in range(world)]
        torch.distributed.all_gather(gathered, stats)
        per_rank = [g.cpu().tolist() for g in gathered]
    else:
        per_rank = [stats.cpu().tolist()]
    wall_max = max(p[0] for p in per_rank)
    value = sum(p[1] for p in per_rank) / wall_max * args.steps / 1e9
    achieved = alg_bytes / (gpu_ms / 1e3) / 1e9
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_t2j(flat, side, h_thrift, toff, opts)
    traffic = None
    tp = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tp):
        with open(tp) as fh:
            traffic = json.load(fh).get("hbm_bytes_per_launch")
    if rank == 0:
        line = {
            "metric": T2J_METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(wall_max / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": CONFIGS[args.config][0], "global_batch": meta["global_batch"], "msgs_per_rank": n,
                       "avg_thrift_bytes": round(thrift_bytes / max(n, 1), 1), "json_bytes_rank0": json_out,
                       "msgs_per_s": round(sum(p[2] for p in per_rank) * args.steps / wall_max), "opts": opts,
                       "ok_msgs_rank0": ok, "checked_vs_oracle": checked,
                       "parallelism": f"dp{world} (one batch per rank), no data-path collective",
                       "per_rank_kernel_ms": [round(p[3], 5) for p in per_rank], "inflight": depth,
                       "serial_gbs": round(sum(p[1] for p in per_rank) / max(p[3] for p in per_rank) / 1e6, 3)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "kernel_ms": round(gpu_ms, 5), "kernel_ms_note": "one batch at a time (serial leg), every launch of the step",
                         "alg_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist:
        torch.distributed.destroy_process_group()
    ctx.close()


# ---------------------------------------------------------------- aggregator
# (threads, calls in flight per thread); the first is `value`. Each thread's part
# of one device batch holds a quarter of its window, so a thread has calls in
# four batches at once (one filling, three converting or coming back).
AGG_RUNS = ((16, 8192), (64, 2048), (64, 1))
# the gateway shape (dg_agg_gateway_drive): logical callers with ONE call in
# flight each (goroutines in Do) over GATEWAY_WORKERS OS threads (the 16
# CPUs a GPU gets) and one dg_agg_wait_gen poller; (callers, depth)
GATEWAY_RUNS = ((1024, 2), (4096, 3), (16384, 4), (65536, 4))
GATEWAY_FILL_DIV = 4  # min_fill = callers / 4: a batch waits for a quarter of the callers (or max_wait); r5y8: 4 > 8 > 16 at 16384
GATEWAY_WORKERS = int(os.environ.get("DG_BENCH_GW_WORKERS", "16"))


def agg_profile(pr, pr0, nbatches, ncalls):
    """dg_agg_profile's counters over a run: us per batch in each stage, ns per call"""
    pr = [pr[i] - pr0[i] for i in range(16)]
    nb_ = max(1, nbatches)
    prof = {k: round(pr[i] / nb_ / 1e3, 1) for i, k in enumerate(
        ("flusher_wait_seal", "flusher_wait_free", "flusher_issue", "completer_wait_hdr", "completer_wait_data",
         "seal_to_issued", "issued_to_done", "callers_blocked"))}
    ncalls = max(1, ncalls)
    prof["ns_per_call_in_submit"] = round(pr[8] / ncalls, 1)
    prof["ns_per_call_in_wait"] = round(pr[9] / ncalls, 1)
    prof["submits_without_open_batch"] = int(pr[10])
    prof["calls_converted_alone"] = int(pr[11])
    for i, k in enumerate(("issue_wait_writers", "issue_buffers", "issue_gather", "issue_convert")):
        prof[k] = round(pr[12 + i] / nb_ / 1e3, 1)
    return prof


def bench_agg(args, rank, world, dev, dist, backend, td, arena, off, meta):
    """The drop-in path: every message is one BinaryConv.Do call (dg_agg
    submit + wait) from `threads` OS threads, as the reference's
    b.RunParallel benchmark does from goroutines (conv/j2t/conv_timing_test.go:
    76-99); the aggregator coalesces them into device batches (upload,
    convert, pack, download overlapped over the ring's 16 batches). A step is
    one pass over all calls; wall-clock timed, host memory in and out."""
    import torch
    import ctypes as C
    from dynamicgo_amd import _lib, conv
    from dynamicgo_amd.thrift import flatten
    flat = flatten(td)
    flags = 1
    L = _lib.lib()
    ctx = conv.Context(dev.index)
    dh = ctx.desc(flat)
    n = len(off) - 1
    lens = np.diff(off).astype(np.uint64)
    out_off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens * 4 + 128, out=out_off[1:])
    out = np.zeros(int(out_off[-1]) + 64, dtype=np.uint8)
    out_len = np.zeros(n, dtype=np.uint64)
    rets = np.zeros(n, dtype=np.uint64)
    lat = np.zeros(n, dtype=np.uint32)
    max_wait_us = 200
    runs = []
    for ri, (threads, window) in enumerate(AGG_RUNS):
        per_thread = max(64, window // int(os.environ.get("DG_BENCH_AGG_SHARE_DIV", "4")))
        if ri == 0:
            max_batch = per_thread
        h = C.c_void_p()
        _lib.check(L.dg_agg_create2(ctx.h, dh, flat.root_type, flags, per_thread, per_thread * 256, max_wait_us,
                                    C.byref(h)))
        secs = C.c_double(0)

        def step(m=n):
            _lib.check(L.dg_agg_drive(h, arena.ctypes.data, off.ctypes.data, m, threads, window, out.ctypes.data,
                                      out_off.ctypes.data, out_len.ctypes.data, rets.ctypes.data, lat.ctypes.data,
                                      C.byref(secs)))
            return secs.value
        m = n if window > 1 else min(n, 16384)  # one call in flight per thread: latency-bound, a shorter pass
        for _ in range(max(1, args.warmup // 2)):
            step(m)
        # the profile counts from here: buffer growth in the warm-up is not the steady state
        b0, tot0, pr0 = C.c_uint64(0), C.c_uint64(0), (C.c_uint64 * 16)()
        _lib.check(L.dg_agg_stats(h, C.byref(b0), C.byref(tot0)))
        _lib.check(L.dg_agg_profile(h, pr0, 16))
        steps = args.steps if ri == 0 else max(2, args.steps // 4)
        if dist:
            torch.distributed.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            step(m)
        wall = time.perf_counter() - t0
        if dist:
            torch.distributed.barrier()
        b = C.c_uint64(0)
        tot = C.c_uint64(0)
        _lib.check(L.dg_agg_stats(h, C.byref(b), C.byref(tot)))
        pr = (C.c_uint64 * 16)()
        _lib.check(L.dg_agg_profile(h, pr, 16))
        prof = agg_profile(pr, pr0, b.value - b0.value, tot.value - tot0.value)
        L.dg_agg_destroy(h)
        lt = lat[:m][lat[:m] > 0].astype(np.float64) / 1e3  # every 8th call is timed (dg_agg_drive)
        runs.append({"threads": threads, "in_flight_per_thread": window, "per_thread_batch_share": per_thread,
                     "calls_per_step": m, "steps": steps,
                     "msgs_per_s": round(m * steps / wall), "gbs_json_in": round(int(off[m]) * steps / wall / 1e9, 3),
                     "ms_per_step": round(wall / steps * 1e3, 3),
                     "lat_us_p50": round(float(np.percentile(lt, 50)), 1),
                     "lat_us_p99": round(float(np.percentile(lt, 99)), 1),
                     "avg_batch": round((tot.value - tot0.value) / max(1, b.value - b0.value), 1), "wall_s": round(wall, 3),
                     "us_per_batch": prof})
        if ri == 0:
            value_wall, value_steps = wall, steps
            # what came back is the reference's output, call by call (outside the timed loop)
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle  # checker only
            chk = oracle.RefOracle() or oracle.PortOracle()
            u = meta.get("unique", n)
            er, eo = chk.j2t_arena(flat, arena, off[:u + 1], flags, nthreads=min(CPU_SHARE, os.cpu_count() or 1))
            bad = 0
            for i in range(n):
                g = i % u
                got = out[int(out_off[i]):int(out_off[i]) + int(out_len[i])].tobytes()
                if int(rets[i]) != int(er[g]) or got != eo[g]:
                    bad += 1
            if bad:
                raise RuntimeError(f"agg: {bad} calls differ from the oracle")
    gw_runs = []
    for callers, depth in GATEWAY_RUNS:
        if os.environ.get("DG_BENCH_NO_GATEWAY"):
            break
        share = max(256, callers // GATEWAY_WORKERS)
        h = C.c_void_p()
        _lib.check(L.dg_agg_create2(ctx.h, dh, flat.root_type, flags, share, share * 256, max_wait_us, C.byref(h)))
        _lib.check(L.dg_agg_set_knob(h, b"depth", depth))
        fill = int(os.environ.get("DG_BENCH_GW_FILL_DIV", GATEWAY_FILL_DIV))
        if fill > 0:
            _lib.check(L.dg_agg_set_knob(h, b"min_fill", callers // fill))
        secs = C.c_double(0)
        st = np.zeros(8, dtype=np.uint64)
        # at least 16 calls per caller in a step: with 65 536 callers the
        # arena's 262 144 calls are 4 per caller, and the step is mostly the
        # callers' ramp and drain (r6z: mean 26 M vs best step 41 M calls/s)
        reps = max(1, callers * 16 // n)
        if reps > 1:
            body = int(off[n])
            ga = np.concatenate([arena[:body]] * reps + [np.zeros(64, dtype=np.uint8)])
            go = np.concatenate([off[:n] + k * body for k in range(reps)] + [np.array([reps * body], dtype=off.dtype)])
            gl = np.diff(go).astype(np.uint64)
            goo = np.zeros(len(go), dtype=np.uint64)
            np.cumsum(gl * 4 + 128, out=goo[1:])
            gout = np.zeros(int(goo[-1]) + 64, dtype=np.uint8)
            gol, grets, glat = (np.zeros(len(gl), dtype=t) for t in (np.uint64, np.uint64, np.uint32))
        else:
            ga, go, goo, gout, gol, grets, glat = arena, off, out_off, out, out_len, rets, lat
        m = n * reps

        def gstep():
            _lib.check(L.dg_agg_gateway_drive(h, ga.ctypes.data, go.ctypes.data, m, GATEWAY_WORKERS, callers,
                                              gout.ctypes.data, goo.ctypes.data, gol.ctypes.data,
                                              grets.ctypes.data, glat.ctypes.data, C.byref(secs), st.ctypes.data))
            return secs.value
        gstep()
        b0, tot0, pr0 = C.c_uint64(0), C.c_uint64(0), (C.c_uint64 * 16)()
        _lib.check(L.dg_agg_stats(h, C.byref(b0), C.byref(tot0)))
        _lib.check(L.dg_agg_profile(h, pr0, 16))
        gsteps = max(2, args.steps // 4)
        ws = [gstep() for _ in range(gsteps)]
        b, tot, pr = C.c_uint64(0), C.c_uint64(0), (C.c_uint64 * 16)()
        _lib.check(L.dg_agg_stats(h, C.byref(b), C.byref(tot)))
        _lib.check(L.dg_agg_profile(h, pr, 16))
        gprof = agg_profile(pr, pr0, b.value - b0.value, tot.value - tot0.value)
        L.dg_agg_destroy(h)
        u = meta.get("unique", n)
        bad = int(sum(1 for i in range(0, m, 97) if int(grets[i]) != 0))
        lt = glat[:m][glat[:m] > 0].astype(np.float64) / 1e3
        gw_runs.append({"callers": callers, "os_threads": GATEWAY_WORKERS, "depth": depth, "per_thread_batch_share": share,
                        "min_fill": callers // fill if fill > 0 else 0,
                        "calls_per_step": m, "steps": gsteps, "msgs_per_s": round(m * gsteps / sum(ws)),
                        "msgs_per_s_best": round(m / min(ws)),
                        "lat_us_p50": round(float(np.percentile(lt, 50)), 1),
                        "lat_us_p99": round(float(np.percentile(lt, 99)), 1),
                        "avg_batch": round((tot.value - tot0.value) / max(1, b.value - b0.value), 1),
                        "parks": int(st[0]), "retries": int(st[1]), "sampled_nonzero_status": bad,
                        "worker_ns_per_call": {k: round(int(st[4 + i]) / max(1, m), 1) for i, k in
                                               enumerate(("in_wait", "in_submit", "idle", "all"))},
                        "us_per_batch": gprof})
    main = runs[0]
    json_bytes = int(off[-1])
    stats = torch.tensor([value_wall, float(json_bytes), float(n)], dtype=torch.float64,
                         device=dev if backend == "nccl" else "cpu")
    if dist:
        gathered = [torch.zeros_like(stats) for _ in range(world)]
        torch.distributed.all_gather(gathered, stats)
        per_rank = [g.cpu().tolist() for g in gathered]
    else:
        per_rank = [stats.cpu().tolist()]
    wall_max = max(p[0] for p in per_rank)
    value = sum(p[2] for p in per_rank) * value_steps / wall_max
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        u = meta.get("unique", n)
        cpu = cpu_baseline(flat, arena[:int(off[u]) + 64], off[:u + 1], flags)
        if cpu:
            cpu["unit"] = "calls/s"
            cpu["value_gbs"], cpu["value"] = cpu["value"], cpu["msgs_per_s"]
    if rank == 0:
        line = {
            "metric": AGG_METRIC, "value": round(value), "unit": "calls/s", "n_gpus": world, "steps": value_steps,
            "warmup": args.warmup, "ms_per_step": round(wall_max / value_steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": CONFIGS[args.config][0], "global_batch": meta["global_batch"], "msgs_per_rank": n,
                       "avg_json_bytes": round(json_bytes / max(n, 1), 1), "flags": flags,
                       "per_thread_batch_share": max_batch, "max_wait_us": max_wait_us, "batches_in_flight": int(os.environ.get("DG_AGG_RING", "8")),
                       "gbs_json_in": main["gbs_json_in"], "lat_us_p50": main["lat_us_p50"],
                       "lat_us_p99": main["lat_us_p99"], "runs": runs, "checked_vs_oracle": n,
                       "gateway_runs": gw_runs,
                       "gateway_note": "callers with one Do in flight each (goroutines) over 16 OS threads, woken per "
                                       "converted generation by one dg_agg_wait_gen poller (INTEGRATION.md §2); "
                                       "compare msgs_per_s with cpu_baseline.share.msgs_per_s (16 cores, same run)",
                       "reference_per_core_ns_per_op": (cpu or {}).get("one_core_ns_per_msg"),
                       "parallelism": f"dp{world} (one aggregator per rank), no data-path collective"},
            "roofline": None,
            "roofline_note": "host path: bound by the host link (H2D of the JSON, D2H of the Thrift) and the "
                             "callers' copies, not by a kernel; the kernels' rooflines are in the c2 line",
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist:
        torch.distributed.destroy_process_group()
    ctx.close()


# ---------------------------------------------------------------- main
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 100 steps: the timed region's fixed cost (the synchronize on each side,
    # the first launch, the in-flight ramp) is ~40-100 us; C2 (r8m, one box):
    # 348.8 / 380.7 / 401.7 GB/s at 20 / 50 / 100 steps of ~32 us
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory end-to-end measurement")
    ap.add_argument("--inflight", type=int, default=None,
                    help="j2t configs: batches in flight in the timed steps (dg_j2t_batch_device_inflight; default "
                         "2, C5's 1M batch 1); the serial (1) rate is reported beside it")
    args = ap.parse_args(argv)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, argv))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    # the batch is built on the CPU before anything touches the GPU (fork pool)
    cpus = max(1, min(CPU_SHARE // max(1, world) or 1, len(os.sched_getaffinity(0))))
    td, arena, off, meta = rank_workload(args.config, rank, world, workers=max(cpus, 2))

    import torch
    ndev = torch.cuda.device_count()
    if ndev == 0:
        raise SystemExit("bench.py needs an MI355X (no HIP device visible)")
    dev = torch.device("cuda", local % ndev)
    torch.cuda.set_device(dev)
    backend = os.environ.get("DG_DIST_BACKEND", "nccl" if ndev >= world else "gloo")
    # DG_FORCE_DIST=1: the distributed branch at world size 1 as well (the
    # RCCL leg on a one-GPU box: tests/test_gpu_dist.py)
    dist = world > 1 or os.environ.get("DG_FORCE_DIST") == "1"
    if dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": dev} if backend == "nccl" else {}
        torch.distributed.init_process_group(backend, rank=rank, world_size=world, **kw)
        if args.config == "c5":  # every rank holds its shard: drop the node's shared copy
            torch.distributed.barrier()
            if local == 0:
                release_c5_cache()

    if args.config.startswith("t2j-"):
        return bench_t2j(args, rank, world, dev, dist, backend, td, arena, off, meta)
    if args.config == "agg":
        return bench_agg(args, rank, world, dev, dist, backend, td, arena, off, meta)

    from dynamicgo_amd import _lib, conv
    from dynamicgo_amd.thrift import flatten
    import ctypes as C
    flat = flatten(td)
    flags = FLAGS.get(args.config, 1)
    L = _lib.lib()
    ctx = conv.Context(dev.index)
    if dist:  # descriptor: built on rank 0, broadcast, created from device memory
        blob = share_descriptor(flat, rank, dev, backend)
        h = C.c_void_p()
        _lib.check(L.dg_desc_create_device(ctx.h, blob.data_ptr(), blob.numel(), C.byref(h)))
        ctx._descs[flat.blob] = h
    dh = ctx.desc(flat)

    n = len(off) - 1
    lens = np.diff(off).astype(np.int64)
    max_len = int(lens.max()) if n else 0  # known to the host that built the arena (dg_j2t_batch_device_ml)
    slots = np.zeros(n + 1, dtype=np.int64)
    np.cumsum((lens * 4 + 64 + 127) & ~127, out=slots[1:])  # dg_slot_bound: 128-byte slots (whole L2 lines)
    d_json = torch.from_numpy(arena).to(dev)
    d_in = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_out = torch.empty(int(slots[-1]) + 64, dtype=torch.uint8, device=dev)
    d_oo = torch.from_numpy(slots).to(dev)
    d_ol = torch.zeros(n, dtype=torch.int32, device=dev)
    d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
    d_pend = torch.zeros(4, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)  # the kernels and the timing events share it
    torch.cuda.set_stream(stream)
    # a 64K batch leaves CUs idle in its tail and list pass that the next
    # batch fills; C5's 1M-message batch does not (measured: 2 in flight 4.73
    # vs 4.45 ms per step)
    depth = max(1, min(8, args.inflight if args.inflight is not None else DEFAULT_INFLIGHT.get(args.config, 2)))
    # one output set per batch in flight (set 0 = the serial leg's buffers)
    osets = [(d_out, d_ol, d_ret, d_pend)] + [
        (torch.empty_like(d_out), torch.zeros_like(d_ol), torch.zeros_like(d_ret), torch.zeros_like(d_pend))
        for _ in range(depth - 1)]
    sets_arr = (C.c_void_p * (4 * depth))(*[t.data_ptr() for o in osets for t in o])

    def step(k=1):
        # k complete batch conversions enqueued by one C call: the step loop
        # runs where a production host (Go via cgo, or C) runs it, not in the
        # Python interpreter (~6 us of ctypes/launch overhead per call)
        _lib.check(L.dg_j2t_batch_device_iters(ctx.h, dh, flat.root_type, d_json.data_ptr(), d_in.data_ptr(), n,
                                               flags, d_out.data_ptr(), d_oo.data_ptr(), d_ol.data_ptr(),
                                               d_ret.data_ptr(), d_pend.data_ptr(), stream.cuda_stream, max_len, k))

    def step_inflight(k):
        # k complete conversions, `depth` of them in flight on the context's
        # streams (forked from / joined into `stream`), set j's buffers each
        _lib.check(L.dg_j2t_batch_device_inflight(ctx.h, dh, flat.root_type, d_json.data_ptr(), d_in.data_ptr(), n,
                                                  flags, d_oo.data_ptr(), sets_arr, depth, stream.cuda_stream,
                                                  max_len, k))

    ctx.stats(reset=True)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    bails, deeps = ctx.stats(reset=True)
    rets = d_ret.cpu().numpy()
    ok = int((rets == 0).sum())
    if int(d_pend.sum().item()) != 0 or ok != n:
        print(f"[rank {rank}] WARNING: {n - ok} messages not ok", file=sys.stderr)
    json_bytes = int(off[-1])
    thrift_bytes = int(d_ol.to(torch.int64).sum().item())
    alg_bytes = json_bytes + thrift_bytes + PER_MSG_META * n
    # the algorithmic bytes of the messages each kernel converts: the wave
    # kernel takes messages longer than the wave_min knob, the first kernel
    # (flat / small / lane) the rest (declines to the list pass are counted
    # with the kernel that listed them: exact_path_msgs_per_step is ~0)
    wmin = C.c_int64(0)
    _lib.check(L.dg_ctx_get_knob(ctx.h, b"wave_min", C.byref(wmin)))
    big = lens > wmin.value
    ol_np = d_ol.cpu().numpy().astype(np.int64)
    route_bytes = [int(lens[~big].sum() + ol_np[~big].sum() + PER_MSG_META * int((~big).sum())),
                   int(lens[big].sum() + ol_np[big].sum() + PER_MSG_META * int(big.sum()))]

    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    # serial leg (one batch at a time): the per-launch time the roofline is
    # priced on -- HIP events on the launch stream
    torch.cuda.synchronize()
    ev0.record(stream)
    step(args.steps)
    ev1.record(stream)
    torch.cuda.synchronize()
    gpu_ms = ev0.elapsed_time(ev1) / args.steps
    # per-kernel leg: the same serial steps with HIP events around each launch
    # of the step (on the launch stream), for the dominant kernel's roofline
    kms = (C.c_double * 3)()
    _lib.check(L.dg_j2t_batch_device_ktime(ctx.h, dh, flat.root_type, d_json.data_ptr(), d_in.data_ptr(), n, flags,
                                           d_out.data_ptr(), d_oo.data_ptr(), d_ol.data_ptr(), d_ret.data_ptr(),
                                           d_pend.data_ptr(), stream.cuda_stream, max_len, args.steps, kms))
    kernel_ms = list(kms)
    dom = int(np.argmax(kernel_ms[:2]))
    if depth > 1:  # warm the in-flight streams and check every set converted the batch
        step_inflight(args.warmup * depth)
        torch.cuda.synchronize()
        for o in osets[1:]:
            if not (torch.equal(o[2], d_ret) and torch.equal(o[1], d_ol) and same_outputs(d_oo, d_ol, o[0], d_out)):
                raise SystemExit("in-flight output set differs from the serial one")

    # timed region: barrier + synchronize on both sides, max over ranks
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    step_inflight(args.steps)
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    wall = time.perf_counter() - t0
    step_ms = ev0.elapsed_time(ev1) / args.steps
    stats = torch.tensor([wall, float(json_bytes), float(n), gpu_ms, step_ms], dtype=torch.float64,
                         device=dev if backend == "nccl" else "cpu")
    if dist:
        gathered = [torch.zeros_like(stats) for _ in range(world)]
        torch.distributed.all_gather(gathered, stats)
        per_rank = [g.cpu().tolist() for g in gathered]
    else:
        per_rank = [stats.cpu().tolist()]
    wall_max = max(p[0] for p in per_rank)
    total_json = sum(p[1] for p in per_rank)
    total_msgs = sum(p[2] for p in per_rank)
    value = total_json / wall_max * args.steps / 1e9
    achieved = alg_bytes / (gpu_ms / 1e3) / 1e9
    dom_achieved = route_bytes[dom] / (kernel_ms[dom] / 1e3) / 1e9 if kernel_ms[dom] > 0 else 0.0
    flat_route = args.config in ("c1", "c2", "c2x", "c2s", "c5")  # flat root, or C5's wrapped flat members

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(flat, arena, off, flags)
    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e and args.config in ("c2", "c3"):
        e2e = e2e_host_path(L, ctx, dh, flat.root_type, flags, arena, off, dev, flat)
    c1 = None
    if rank == 0 and args.config == "c1":  # BinaryConv.Do latency: one message, host in -> host out
        cv = conv.BinaryConv(conv.Options(), ctx=ctx)
        m = bytes(arena[:int(off[1])])
        for _ in range(20):
            cv.do(flat, m)
        t = []
        for _ in range(200):
            t0 = time.perf_counter()
            cv.do(flat, m)
            t.append(time.perf_counter() - t0)
        # the same call straight through the C ABI a cgo binding uses
        # (dg_j2t_do, preallocated output), without the Python mirror's
        # per-call array building
        obuf = C.create_string_buffer(4 * len(m) + 256)
        olen = C.c_size_t(0)
        oret = C.c_uint64(0)
        tc = []
        for k in range(220):
            t0 = time.perf_counter()
            _lib.check(L.dg_j2t_do(ctx.h, dh, flat.root_type, m, len(m), flags, obuf, len(obuf), C.byref(olen),
                                   C.byref(oret)))
            if k >= 20:
                tc.append(time.perf_counter() - t0)
        if oret.value != 0 or obuf.raw[:olen.value] != cv.do(flat, m):
            raise SystemExit("dg_j2t_do differs from BinaryConv.do")
        c1 = {"do_latency_us_median": round(float(np.median(t)) * 1e6, 1),
              "do_latency_c_abi_us_median": round(float(np.median(tc)) * 1e6, 1),
              "note": "one message, host in -> host out, synchronous: BinaryConv.do (the Python mirror: "
                      "dg_j2t_batch_host) and dg_j2t_do called directly through ctypes (the C ABI a cgo binding "
                      "calls: one pinned upload, the kernels, the packing, one download)"}

    traffic = None
    tp = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tp):
        with open(tp) as fh:
            traffic = json.load(fh).get("hbm_bytes_per_launch")

    if rank == 0:
        scaling = CONFIGS[args.config][2]
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(wall_max / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": CONFIGS[args.config][0], "global_batch": meta["global_batch"],
                       "msgs_per_rank": n, "avg_json_bytes": round(json_bytes / max(n, 1), 1),
                       "msgs_per_s": round(total_msgs * args.steps / wall_max),
                       "thrift_bytes_rank0": thrift_bytes, "flags": flags,
                       "parallelism": f"dp{world} ({'byte-balanced shards of one batch' if scaling == 'strong' else 'one batch per rank'}, "
                                      f"descriptor broadcast over {backend if dist else '-'}), no data-path collective",
                       "ok_msgs_rank0": ok,
                       "exact_path_msgs_per_step": bails / max(1, args.warmup),
                       "deep_msgs_per_step": deeps / max(1, args.warmup),
                       "per_rank_gbs": [round(p[1] / p[0] * args.steps / 1e9, 3) for p in per_rank],
                       "per_rank_kernel_ms": [round(p[3], 5) for p in per_rank],
                       "inflight": depth,
                       "per_rank_inflight_step_ms": [round(p[4], 5) for p in per_rank],
                       "serial_gbs": round(total_json / max(p[3] for p in per_rank) / 1e6, 3)},
            "roofline": {"bound": "hbm", "achieved": round(dom_achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(dom_achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "traffic_source": f"profiles/traffic_{args.config}.json (PMC, committed)" if traffic else None,
                         "kernel": KERNEL_NAMES[dom][0 if flat_route else 1] if dom == 0 else KERNEL_NAMES[1],
                         "kernel_ms": round(kernel_ms[dom], 5),
                         "alg_bytes_per_launch": route_bytes[dom],
                         "kernel_ms_note": "the dominant kernel's average launch, HIP events on its launch stream "
                                           "(dg_j2t_batch_device_ktime, serial leg); alg bytes = JSON + Thrift + 28 "
                                           "per message it converts",
                         "per_kernel_ms": {"first": round(kernel_ms[0], 5), "wave": round(kernel_ms[1], 5),
                                           "list_pass": round(kernel_ms[2], 5)},
                         "step": {"achieved": round(achieved, 2), "frac": round(achieved / HBM_PEAK_GBS, 5),
                                  "ms": round(gpu_ms, 5), "alg_bytes": alg_bytes,
                                  "note": "every launch of the serial step (incl. list pass and launch gaps)"}},
            "cpu_baseline": cpu,
        }
        if e2e is not None:
            line["e2e_host"] = e2e
        if c1 is not None:
            line["c1"] = c1
        print(json.dumps(line), flush=True)
    if dist:
        torch.distributed.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
