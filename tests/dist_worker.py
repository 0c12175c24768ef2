"""One rank of the multi-GPU path, run as a child process by
tests/test_gpu_dist.py: bench.py's own rank code on the GPU, checked against
the oracle.

    python tests/dist_worker.py BACKEND RESULT_DIR

with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the
environment. The rank joins the process group exactly as bench.main() does
(nccl: init_process_group(device_id=...)), takes its byte-balanced shard of a
reduced C5 batch (bench.rank_workload), receives rank 0's flattened
descriptor over the backend (bench.share_descriptor: RCCL broadcast straight
into device memory under nccl), creates the device descriptor from that
device buffer (dg_desc_create_device), converts its shard on the GPU and
compares every message with the oracle. It writes RESULT_DIR/rank<r>.json.
Test infrastructure only (it imports oracle/)."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

C5_N, C5_SCALE = 3000, 0.05


def main():
    backend, out_dir = sys.argv[1], sys.argv[2]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    import bench
    td, a, off, meta = bench.rank_workload("c5", rank, world, c5_n=C5_N, c5_scale=C5_SCALE)
    import numpy as np
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    kw = {"device_id": dev} if backend == "nccl" else {}
    dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    res = {"rank": rank, "world": world, "backend": backend, "shard": meta["shard"]}
    try:
        dist.barrier()
        if local == 0:
            bench.release_c5_cache(C5_N, 45, C5_SCALE)
        from dynamicgo_amd import _lib, conv, thrift as T
        flat = T.flatten(td)
        sent = flat if rank == 0 else T.FlatDescriptor(b"", flat.root_type, flat.types)
        blob = bench.share_descriptor(sent, rank, dev, backend)
        res["blob_on_device"] = blob.device.type == "cuda"
        res["blob_equal"] = bytes(blob.cpu().numpy().tobytes()) == flat.blob
        ctx = conv.Context(dev.index)
        L = _lib.lib()
        h = C.c_void_p()
        _lib.check(L.dg_desc_create_device(ctx.h, blob.data_ptr(), blob.numel(), C.byref(h)))
        ctx._descs[flat.blob] = h  # the broadcast descriptor, not a fresh host upload
        n = len(off) - 1
        msgs = [bytes(a[int(off[i]):int(off[i + 1])]) for i in range(n)]
        outs, rets = conv.BinaryConv(conv.Options(), ctx=ctx).do_batch(flat, msgs)
        import oracle
        chk = oracle.RefOracle() or oracle.PortOracle()
        wr, wo = chk.j2t_arena(flat, np.ascontiguousarray(a), off, 1)
        bad = [i for i in range(n) if int(rets[i]) != int(wr[i]) or (int(wr[i]) == 0 and outs[i] != wo[i])]
        res.update(n=n, mismatches=len(bad), first_bad=bad[:5], ok=int((np.asarray(rets) == 0).sum()))
        # the stats exchange bench.py does after its timed region
        stats = torch.tensor([float(n)], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        got = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(got, stats)
        res["gathered_n"] = [int(g.item()) for g in got]
        ctx.close()
    finally:
        dist.destroy_process_group()
    with open(os.path.join(out_dir, "rank%d.json" % rank), "w") as fh:
        json.dump(res, fh)


if __name__ == "__main__":
    main()
