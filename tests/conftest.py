import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


class _Flat:
    def __init__(self, blob, root):
        self.blob = blob
        self.root_type = root


@pytest.fixture(scope="session")
def golden():
    """(rows, flats): the reference-generated fixtures."""
    with open(os.path.join(GOLDEN, "descs.json")) as fh:
        d = json.load(fh)
    flats = {k: _Flat(bytes.fromhex(v["blob"]), v["root"]) for k, v in d.items()}
    rows = []
    with open(os.path.join(GOLDEN, "j2t_golden.jsonl")) as fh:
        for line in fh:
            r = json.loads(line)
            rows.append((r["desc"], r["flags"], bytes.fromhex(r["json"]), r["ret"], bytes.fromhex(r["out"])))
    return rows, flats


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture
def knob():
    """knob(name, value): set a routing knob of the default context
    (dg_ctx_set_knob); every knob touched is restored after the test."""
    from dynamicgo_amd import conv
    ctx = conv.default_context()
    saved = {}

    def set_(name, value):
        if name not in saved:
            saved[name] = ctx.get_knob(name)
        ctx.set_knob(name, int(value))

    yield set_
    for k, v in saved.items():
        ctx.set_knob(k, v)


# The full C5 batch (1 048 576 messages, seed 45) for tests/test_gpu_full.py:
# generated with a fork pool right after collection, before any test has
# touched the GPU (a process that initialised HIP must not fork workers).
_C5 = {}


def pytest_collection_finish(session):
    if not any("test_full_c5_batch" in it.nodeid for it in session.items):
        return
    from dynamicgo_amd import workloads as W
    try:
        cpus = len(os.sched_getaffinity(0))
    except AttributeError:
        cpus = os.cpu_count() or 1
    _C5["arena"], _C5["off"] = W.gen_mixed_arena(1 << 20, 45, workers=max(1, min(16, cpus)))


@pytest.fixture(scope="session")
def c5_batch():
    """(arena, offsets) of the benched C5 batch (bench.py --config c5)."""
    if "arena" not in _C5:
        from dynamicgo_amd import workloads as W
        _C5["arena"], _C5["off"] = W.gen_mixed_arena(1 << 20, 45, workers=1)
    return _C5["arena"], _C5["off"]
