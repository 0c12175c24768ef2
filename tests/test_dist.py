"""The N>1 path on CPU (gloo, world_size 2): descriptor broadcast and
byte-balanced sharding give each rank exactly its messages, and the per-rank
results concatenate to the single-rank result."""
import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from dynamicgo_amd import dist as D, thrift as T, workloads as W


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


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fl = T.flatten(W.simple_desc())
        blob = D.broadcast_blob(fl.blob if rank == 0 else None, torch.device("cpu"))
        got = bytes(blob.numpy().tobytes())
        msgs = W.gen_flat_batch(random.Random(42), 600)
        a, off = W.arena(msgs)
        lo, hi = D.shard_ranges(off, world)[rank]
        chk = oracle.PortOracle()
        mine = [chk.j2t(T.FlatDescriptor(got, fl.root_type, fl.types), m, 1) for m in msgs[lo:hi]]
        allr = [None] * world
        dist.all_gather_object(allr, (lo, hi, mine))
        if rank == 0:
            q.put((got == fl.blob, allr))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_broadcast_and_shards():
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
    msgs = W.gen_flat_batch(random.Random(42), 600)
    fl = T.flatten(W.simple_desc())
    chk = oracle.PortOracle()
    whole = [chk.j2t(fl, m, 1) for m in msgs]
    cat = []
    for lo, hi, res in sorted(parts, key=lambda x: x[0]):
        cat.extend(res)
    assert parts[0][1] == parts[1][0]
    assert cat == whole
