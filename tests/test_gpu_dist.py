"""The multi-GPU leg on the hardware one box has: bench.py's
distributed setup with the `nccl` (RCCL) backend at world size 1 --
init_process_group(device_id=...), the descriptor broadcast into device
memory, dg_desc_create_device on the received buffer, a reduced C5 shard vs
the oracle -- and two ranks sharing the one GPU over gloo, so the first
8-GPU run is not that code's first execution. Each rank is its own process
(tests/dist_worker.py); the GPU processes stay far below the box's limit."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "dist_worker.py")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(backend, world, tmp_path):
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if world > 1:
            env["LOCAL_RANK"] = "0"  # every rank on the box's one GPU
        procs.append(subprocess.Popen([sys.executable, "-u", WORKER, backend, str(tmp_path)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(out.decode(errors="replace")[-3000:])
    assert all(p.returncode == 0 for p in procs), "\n".join(logs)
    return [json.load(open(os.path.join(tmp_path, "rank%d.json" % r))) for r in range(world)]


def test_nccl_world1_broadcast_and_convert(tmp_path):
    res = _run("nccl", 1, tmp_path)[0]
    assert res["blob_on_device"] and res["blob_equal"]
    assert res["n"] == 3000 and res["mismatches"] == 0, res
    assert res["gathered_n"] == [3000]


def test_gloo_world2_one_gpu_shards_vs_oracle(tmp_path):
    res = _run("gloo", 2, tmp_path)
    assert [r["shard"] for r in res] == [[0, res[0]["shard"][1]], [res[0]["shard"][1], 3000]]
    for r in res:
        assert r["blob_equal"] and r["mismatches"] == 0, r
        assert r["gathered_n"] == [x["n"] for x in res]
    assert sum(r["n"] for r in res) == 3000


def test_bench_nccl_world1_line(tmp_path):
    """bench.py itself through its distributed branch (DG_FORCE_DIST=1) at
    world size 1 over RCCL: every message converts and the line names nccl."""
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_port()), DG_FORCE_DIST="1")
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--config", "c2", "--steps", "3",
                        "--warmup", "1", "--no-cpu-baseline", "--no-e2e"], env=env, capture_output=True, timeout=110)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    line = json.loads(p.stdout.decode().strip().splitlines()[-1])
    cfg = line["config"]
    assert cfg["ok_msgs_rank0"] == cfg["msgs_per_rank"] == 65536
    assert "over nccl" in cfg["parallelism"]
    assert line["n_gpus"] == 1 and line["value"] > 0
