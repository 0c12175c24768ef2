"""ctypes binding of the C ABI (include/dgj2t.h) exported by libdgj2t.so.

The product path has no CPU fallback: if the HIP library is missing or fails
to load, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DG_LIB_PATH") or os.path.join(HERE, "libdgj2t.so")

# symbols include/dgj2t.h declares (checked by tests/test_abi.py)
EXPORTS = ["dg_last_error", "dg_build_info", "dg_ctx_create", "dg_ctx_destroy", "dg_ctx_stream", "dg_ctx_stats", "dg_ctx_counters", "dg_ctx_set_knob", "dg_ctx_get_knob",
           "dg_desc_create",
           "dg_desc_create_device", "dg_desc_destroy", "dg_desc_root", "dg_j2t_batch_device",
           "dg_j2t_batch_device_ml", "dg_j2t_batch_device_hm", "dg_j2t_batch_device_cb", "dg_j2t_batch_device_iters",
           "dg_j2t_batch_device_inflight", "dg_j2t_batch_device_ktime",
           "dg_slot_bound", "dg_j2t_batch_host", "dg_j2t_batch_host_hm", "dg_j2t_batch_host_cb", "dg_j2t_do", "dg_pack_device", "dg_pack_device_scan", "dg_pack_device_framed", "dg_agg_create", "dg_agg_create2", "dg_agg_do",
           "dg_agg_submit", "dg_agg_wait", "dg_agg_ready", "dg_agg_stats", "dg_agg_profile", "dg_agg_destroy", "dg_agg_drive", "dg_agg_wait_gen", "dg_agg_ticket_gen", "dg_agg_set_knob",
           "dg_agg_gateway_drive", "dg_j2t_pipeline_host", "dg_bench_device", "dg_desc_attach_t2j", "dg_t2j_slot_bound", "dg_t2j_batch_device", "dg_t2j_batch_device_ml",
           "dg_t2j_batch_host", "dg_t2j_batch_device_aux", "dg_t2j_batch_host_aux",
           "dg_t2j_batch_device_cb", "dg_t2j_batch_host_cb"]

_lib = None


class DGError(RuntimeError):
    pass


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise DGError(f"{LIB_PATH} missing: the HIP transcoder is not built "
                      "(run __graft_entry__.build() or python -m dynamicgo_amd.build)")
    # One HIP runtime per process: torch ships its own libamdhip64 (soname
    # libamdhip64.so.7, file libamdhip64.so). Loading torch first makes our
    # NEEDED libamdhip64.so.7 resolve to that copy instead of a second runtime.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    L = C.CDLL(LIB_PATH)
    vp, u32, u64, sz, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_size_t, C.c_int
    P64 = C.POINTER(C.c_uint64)
    sig = {
        "dg_last_error": (C.c_char_p, []),
        "dg_build_info": (C.c_char_p, []),
        "dg_ctx_create": (i32, [i32, C.POINTER(vp)]),
        "dg_ctx_destroy": (None, [vp]),
        "dg_ctx_stream": (vp, [vp]),
        "dg_ctx_stats": (i32, [vp, P64, P64, i32]),
        "dg_ctx_counters": (i32, [vp, P64, i32, i32]),
        "dg_ctx_set_knob": (i32, [vp, C.c_char_p, C.c_int64]),
        "dg_ctx_get_knob": (i32, [vp, C.c_char_p, C.POINTER(C.c_int64)]),
        "dg_desc_create": (i32, [vp, C.c_char_p, sz, C.POINTER(vp)]),
        "dg_desc_create_device": (i32, [vp, vp, sz, C.POINTER(vp)]),
        "dg_desc_destroy": (None, [vp]),
        "dg_desc_root": (u32, [vp]),
        "dg_j2t_batch_device": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, vp, vp, vp, vp, vp]),
        "dg_j2t_batch_device_ml": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, vp, vp, vp, vp, vp, u64]),
        "dg_j2t_batch_device_hm": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, u32, vp, vp, vp, vp, vp, vp, vp, u64]),
        "dg_j2t_batch_host_hm": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, u32, vp, u64, vp, u64, vp, vp, P64]),
        "dg_j2t_batch_device_cb": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, vp, vp, vp, vp, vp, vp, u64]),
        "dg_j2t_batch_host_cb": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, vp, u64, vp, vp, P64]),
        "dg_j2t_batch_device_iters": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, vp, vp, vp, vp, vp, u64, C.c_int]),
        "dg_j2t_batch_device_ktime": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, vp, vp, vp, vp, vp, u64, C.c_int,
                                           C.POINTER(C.c_double)]),
        "dg_j2t_batch_device_inflight": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, vp, C.c_int, vp, u64, C.c_int]),
        "dg_slot_bound": (u64, [u64]),
        "dg_j2t_batch_host": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, u64, vp, vp, P64]),
        "dg_j2t_do": (i32, [vp, vp, u32, C.c_char_p, sz, u64, vp, sz, C.POINTER(sz), P64]),
        "dg_pack_device": (i32, [vp, vp, vp, vp, u64, vp, vp, vp]),
        "dg_pack_device_scan": (i32, [vp, vp, vp, vp, u64, vp, vp, vp]),
        "dg_pack_device_framed": (i32, [vp, vp, vp, vp, vp, u64, C.c_char_p, u32, C.c_char_p, u32, vp, vp, vp]),
        "dg_agg_create": (i32, [vp, vp, u32, u64, u32, u32, C.POINTER(vp)]),
        "dg_agg_do": (i32, [vp, C.c_char_p, sz, vp, sz, C.POINTER(sz), P64]),
        "dg_agg_create2": (i32, [vp, vp, u32, u64, u32, u64, u32, C.POINTER(vp)]),
        "dg_agg_submit": (i32, [vp, C.c_char_p, sz, i32, vp]),
        "dg_agg_wait": (i32, [vp, vp, vp, sz, C.POINTER(sz), P64]),
        "dg_agg_ready": (i32, [vp, vp]),
        "dg_agg_drive": (i32, [vp, vp, vp, u64, i32, i32, vp, vp, vp, vp, vp, C.POINTER(C.c_double)]),
        "dg_agg_wait_gen": (i32, [vp, u64, u32, P64]),
        "dg_agg_ticket_gen": (u64, [vp]),
        "dg_agg_set_knob": (i32, [vp, C.c_char_p, C.c_int64]),
        "dg_agg_gateway_drive": (i32, [vp, vp, vp, u64, i32, i32, vp, vp, vp, vp, vp, C.POINTER(C.c_double), vp]),
        "dg_j2t_pipeline_host": (i32, [vp, vp, u32, vp, vp, u64, u64, u32, vp, u64, vp, vp, P64]),
        "dg_agg_stats": (i32, [vp, P64, P64]),
        "dg_agg_profile": (i32, [vp, P64, i32]),
        "dg_agg_destroy": (None, [vp]),
        "dg_desc_attach_t2j": (i32, [vp, C.c_char_p, sz]),
        "dg_t2j_slot_bound": (u64, [u64]),
        "dg_t2j_batch_device": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, vp, vp, vp, vp]),
        "dg_t2j_batch_device_ml": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, vp, vp, vp, vp, u64]),
        "dg_t2j_batch_host": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, u64, vp, vp, P64]),
        "dg_t2j_batch_device_aux": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, vp, vp, vp, vp, vp, u64]),
        "dg_t2j_batch_host_aux": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, u64, vp, vp, P64, vp]),
        "dg_t2j_batch_device_cb": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, vp, vp, vp, vp, vp, vp, vp, u64]),
        "dg_t2j_batch_host_cb": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, u64, vp, vp, P64, vp, vp]),
        "dg_bench_device": (i32, [vp, vp, u32, vp, vp, u64, u64, vp, vp, vp, vp, i32, C.POINTER(C.c_float)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _check_provenance(L)
    _lib = L
    return L


BUILD_INFO = None


def _check_provenance(L):
    """The loaded library must be built from the sources next to it (the
    hash build.py compiles in); a stale or foreign binary fails loudly."""
    global BUILD_INFO
    BUILD_INFO = L.dg_build_info().decode()
    got = BUILD_INFO.split(":", 1)[1].split()[0] if ":" in BUILD_INFO else "?"
    try:
        from .build import source_hash
        want = source_hash()
    except OSError:  # sources not shipped: nothing to compare against
        want = got
    if got != want and not os.environ.get("DG_ALLOW_STALE"):
        raise DGError(f"{LIB_PATH} was built from other sources ({got}, sources here: {want}); "
                      "rebuild with python -m dynamicgo_amd.build")
    if os.environ.get("DG_LOG_LIB"):
        import sys
        print(f"[dynamicgo_amd] loaded {LIB_PATH} ({BUILD_INFO})", file=sys.stderr, flush=True)


class HMEntry(C.Structure):
    """dg_hm_entry (include/dgj2t_defs.h)"""
    _fields_ = [("off", C.c_uint32), ("len", C.c_uint32), ("mask", C.c_uint64)]


class VMEntry(C.Structure):
    """dg_cb_entry (include/dgj2t_defs.h)"""
    _fields_ = [("off", C.c_uint32), ("count", C.c_uint32)]


class CBTables(C.Structure):
    """dg_cb_tables (include/dgj2t_defs.h)"""
    _fields_ = [("hm_tab", C.c_void_p), ("n_hm", C.c_uint32), ("ans_tab", C.c_void_p),
                ("bytes", C.c_void_p), ("len", C.c_uint64)]


def check(rc: int):
    if rc != 0:
        msg = lib().dg_last_error()
        raise DGError(f"dgj2t error {rc}: {msg.decode() if msg else ''}")
