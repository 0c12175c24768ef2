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


def test_same_outputs_compares_slot_prefixes_in_passes():
    """The in-flight check (bench.same_outputs): every message's slot prefix
    of out_len bytes is compared, the slot tails are not, over more messages
    than one pass takes (C5's 1M messages at depth 2 once ran its masks out
    of memory)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(5)
    n = (1 << 16) * 2 + 123
    lens = rng.integers(0, 40, n)
    oo = np.zeros(n + 1, np.int64)
    np.cumsum((lens + 64 + 7) // 8 * 8, out=oo[1:])
    d_oo, d_ol = torch.from_numpy(oo), torch.from_numpy(lens.astype(np.int32))
    a = torch.from_numpy(rng.integers(0, 256, int(oo[-1]) + 64, dtype=np.uint8))
    b = a.clone()
    assert bench.same_outputs(d_oo, d_ol, a, b)
    k = n - 7
    b[int(oo[k]) + int(lens[k]) + 3] ^= 1  # a slot tail: not compared
    assert bench.same_outputs(d_oo, d_ol, a, b)
    k = int(np.nonzero(lens[(1 << 16) + 5:])[0][0]) + (1 << 16) + 5  # a prefix byte in the second pass
    b[int(oo[k])] ^= 1
    assert not bench.same_outputs(d_oo, d_ol, a, b)
