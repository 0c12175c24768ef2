"""What bench.py's records state, checked on the CPU: the
CPU baseline's core count is the cores that can run at once (the cgroup
quota caps the affinity), per-core figures divide by that count, and the
all-affinity leg is reported beside it; the workload's algorithmic bytes are
split by the kernel that converts them."""
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import oracle  # noqa: E402
from dynamicgo_amd import thrift as T, workloads as W  # noqa: E402


def test_host_cpu_env_reads_quota():
    env = bench.host_cpu_env()
    assert env["affinity_cpus"] >= 1
    assert "quota_cpus" in env  # None when unlimited


@pytest.mark.skipif(oracle.RefOracle() is None, reason="oracle/_ref not built")
def test_cpu_baseline_cores_are_the_quota_bounded_ones(monkeypatch):
    fl = T.flatten(W.simple_desc())
    msgs = W.gen_flat_batch(random.Random(1), 4000)
    arena, off = W.arena(msgs)
    quota = bench.host_cpu_env().get("quota_cpus")
    phys, _ = oracle.physical_cpus()
    want = max(1, min(bench.CPU_SHARE, len(phys), int(quota) if quota else len(phys)))
    cb = bench.cpu_baseline(fl, arena, off, 1, budget_s=0.05)
    assert cb["cores"] == want
    assert cb["kind"] == "reference"
    assert abs(cb["per_core_gbs"] - cb["value"] / cb["cores"]) < 1e-3
    assert cb["all_affinity"]["cores"] == max(1, len(phys))
    assert cb["range"]["min"] <= cb["value"] <= cb["range"]["max"]
    assert cb["range_ratio"] >= 1.0
    # a fake 2-CPU quota caps the count
    real = bench.host_cpu_env
    monkeypatch.setattr(bench, "host_cpu_env", lambda: dict(real(), quota_cpus=2.0))
    cb2 = bench.cpu_baseline(fl, arena, off, 1, budget_s=0.05)
    assert cb2["cores"] == min(2, len(phys))
