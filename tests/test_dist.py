"""The N>1 path on CPU (gloo, world_size 2), driven through bench.py's own
rank code: rank_workload (C5 as ONE batch, byte-balanced shard per rank),
share_descriptor (the broadcast), and spawn_ranks (bench.py --gpus N
launching its ranks). Each rank's shard converted by the oracle concatenates
to the whole batch's result."""
import os
import random
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from dynamicgo_amd import dist as D, thrift as T, workloads as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

C5_N, C5_SCALE = 3000, 0.05


def test_shard_ranges_cover_and_balance():
    rng = random.Random(7)
    msgs = W.gen_flat_batch(rng, 1000) + W.gen_nested_batch(rng, 50)
    _, off = W.arena(msgs)
    for world in (1, 2, 3, 4, 8):
        rs = D.shard_ranges(off, world)
        assert rs[0][0] == 0 and rs[-1][1] == len(msgs)
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
        sizes = [int(off[h] - off[l]) for l, h in rs]
        assert max(sizes) - min(sizes) <= 2 * max(len(m) for m in msgs)
    assert D.shard_ranges(np.array([0], dtype=np.uint64), 4) == [(0, 0)] * 4


def test_c5_generation_is_worker_independent_and_shards_partition():
    a1, o1 = W.gen_mixed_arena(C5_N, 45, workers=1, large_scale=C5_SCALE, chunk=512)
    a2, o2 = W.gen_mixed_arena(C5_N, 45, workers=3, large_scale=C5_SCALE, chunk=512)
    assert (o1 == o2).all() and (a1 == a2).all()
    for world in (1, 2, 4, 8):
        parts = [bench.rank_workload("c5", r, world, c5_n=C5_N, c5_scale=C5_SCALE) for r in range(world)]
        assert all(p[3]["global_batch"] == C5_N for p in parts)
        got = b"".join(bytes(p[1][:int(p[2][-1])]) for p in parts)
        a, o = W.gen_mixed_arena(C5_N, 45, large_scale=C5_SCALE)
        assert got == bytes(a[:int(o[-1])])
        assert sum(len(p[2]) - 1 for p in parts) == C5_N
        bench.release_c5_cache(C5_N, 45, C5_SCALE)
    assert not [f for f in os.listdir("/dev/shm") if f.startswith("dgj2t_c5_")]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        td, a, off, meta = bench.rank_workload("c5", rank, world, c5_n=C5_N, c5_scale=C5_SCALE)
        dist.barrier()
        if rank == 0:  # every rank has its shard: the node's shared copy goes
            bench.release_c5_cache(C5_N, 45, C5_SCALE)
        fl = T.flatten(td)
        blob = bench.share_descriptor(fl if rank == 0 else T.FlatDescriptor(b"", fl.root_type, fl.types), rank,
                                      torch.device("cpu"), "gloo")
        got = bytes(blob.numpy().tobytes())
        chk = oracle.PortOracle()
        rets, outs = chk.j2t_arena(T.FlatDescriptor(got, fl.root_type, fl.types), a, off, 1)
        allr = [None] * world
        dist.all_gather_object(allr, (meta["shard"], [int(r) for r in rets], outs))
        if rank == 0:
            q.put((got == fl.blob, allr))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_bench_rank_path():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        same_blob, parts = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert same_blob
    td, a, off, _ = bench.rank_workload("c5", 0, 1, c5_n=C5_N, c5_scale=C5_SCALE)
    fl = T.flatten(td)
    rets, outs = oracle.PortOracle().j2t_arena(fl, a, off, 1)
    parts = sorted(parts, key=lambda x: x[0][0])
    assert parts[0][0][1] == parts[1][0][0] and parts[0][0][0] == 0 and parts[1][0][1] == C5_N
    assert sum((p[1] for p in parts), []) == [int(r) for r in rets]
    assert sum((p[2] for p in parts), []) == outs


def test_spawn_ranks_sets_the_rank_env(tmp_path):
    """bench.py --gpus N (no WORLD_SIZE) starts N children with the
    torch.distributed env; here the child is a probe script, not the GPU run."""
    probe = tmp_path / "probe.py"
    probe.write_text("import os, sys\n"
                     "open(os.path.join(sys.argv[1], 'r' + os.environ['RANK']), 'w').write("
                     "' '.join(os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR')))\n")
    rc = bench.spawn_ranks(3, [str(tmp_path)], script=str(probe))
    assert rc == 0
    for r in range(3):
        assert (tmp_path / f"r{r}").read_text() == f"{r} {r} 3 127.0.0.1"
