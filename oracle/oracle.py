"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes front-ends for the two CPU checkers under oracle/:

* ``RefOracle``  — oracle/_ref/libdgref.so: the reference's own native/native.c
  compiled unmodified + ref_harness.c (the ground truth; see oracle/Makefile).
* ``PortOracle`` — oracle/_build/libj2t_oracle.so: our plain-C restatement of
  the j2t path (oracle/j2t_oracle.c), pinned against RefOracle and the golden
  fixtures in tests/golden/.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / reported baseline — never as the thing
measured or shipped.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def _cpu_has_avx2() -> bool:
    try:
        with open("/proc/cpuinfo") as fh:
            return " avx2" in fh.read()
    except OSError:
        return False


class _Base:
    def __init__(self, lib: C.CDLL, prefix: str):
        self.lib = lib
        self.p = prefix
        f = getattr(lib, prefix + "desc_create")
        f.restype = C.c_void_p
        f.argtypes = [C.c_char_p, C.c_size_t]
        g = getattr(lib, prefix + "desc_destroy")
        g.argtypes = [C.c_void_p]
        j = getattr(lib, prefix + "j2t")
        j.restype = C.c_uint64
        j.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_size_t, C.c_uint64,
                      C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
        b = getattr(lib, prefix + "j2t_batch")
        b.restype = C.c_int
        b.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64,
                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        self._descs = {}

    def _desc(self, blob: bytes):
        h = self._descs.get(blob)
        if h is None:
            h = getattr(self.lib, self.p + "desc_create")(blob, len(blob))
            if not h:
                raise ValueError("bad descriptor blob")
            self._descs[blob] = h
        return h

    def j2t(self, flat, json: bytes, flags: int, root: Optional[int] = None) -> Tuple[int, bytes]:
        """One message -> (packed ret, thrift bytes); bytes are b"" on error."""
        d = self._desc(flat.blob)
        root = flat.root_type if root is None else root
        cap = 16 * len(json) + 65536
        out = C.create_string_buffer(cap)
        ol = C.c_size_t(0)
        n = len(json)
        # 64 zero bytes after the message: the reference's SIMD advance_string
        # (native/scanning.c:130-375) reads whole blocks past the end of an
        # unterminated string, so without padding its verdict depends on
        # whatever heap bytes follow the Python object (a quote there ends the
        # "string" past the buffer). With zeros it reports ERR_EOF like the port.
        json = bytes(json) + bytes(64)
        ret = getattr(self.lib, self.p + "j2t")(d, root, json, n, flags, out, cap, C.byref(ol))
        if ret != 0:
            return int(ret), b""
        if ol.value > cap:  # the harness reports the full length: once more with room
            cap = ol.value + 64
            out = C.create_string_buffer(cap)
            ret = getattr(self.lib, self.p + "j2t")(d, root, json, n, flags, out, cap, C.byref(ol))
            if ret != 0 or ol.value > cap:
                raise RuntimeError("oracle output exceeded harness capacity")
        return 0, out.raw[:ol.value]

    def j2t_hm(self, flat, json: bytes, flags: int, prefix: bytes, root: Optional[int] = None) -> Tuple[int, bytes]:
        """One message with the root's HTTP-mapped fields written by the host
        as `prefix` (handleHttpMappings emulation, reference harness only)."""
        f = getattr(self.lib, self.p + "j2t_hm")
        f.restype = C.c_uint64
        f.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_size_t, C.c_uint64, C.c_char_p, C.c_size_t,
                      C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
        d = self._desc(flat.blob)
        root = flat.root_type if root is None else root
        cap = 16 * len(json) + len(prefix) + 65536
        out = C.create_string_buffer(cap)
        ol = C.c_size_t(0)
        ret = f(d, root, json, len(json), flags, prefix, len(prefix), out, cap, C.byref(ol))
        if ret != 0:
            return int(ret), b""
        return 0, out.raw[:ol.value]

    def j2t_hm2(self, flat, json: bytes, flags: int, prefix: bytes, mask: int, root: Optional[int] = None):
        """j2t_hm with the host's mask of the mapped fields it wrote (bit k =
        the root's k-th field in id order). Returns (ret, out, field_cache):
        for the root's ERR_HM_END (code 21) `out` is the output so far and
        `field_cache` the unmatched field ids (reference harness only)."""
        f = getattr(self.lib, self.p + "j2t_hm2")
        f.restype = C.c_uint64
        f.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_size_t, C.c_uint64, C.c_char_p, C.c_size_t,
                      C.c_uint64, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t), C.c_void_p, C.c_size_t,
                      C.POINTER(C.c_size_t)]
        d = self._desc(flat.blob)
        root = flat.root_type if root is None else root
        cap = 16 * len(json) + len(prefix) + 65536
        out = C.create_string_buffer(cap)
        ol = C.c_size_t(0)
        fc = (C.c_int32 * 4096)()
        fl = C.c_size_t(0)
        ret = f(d, root, json, len(json), flags, prefix, len(prefix), mask & (2**64 - 1), out, cap, C.byref(ol),
                fc, 4096, C.byref(fl))
        if ret != 0 and (ret & 0xFF) != 21:
            return int(ret), b"", []
        return int(ret), out.raw[:ol.value], [int(fc[k]) for k in range(fl.value)]

    def j2t_hm3(self, flat, json: bytes, flags: int, entries, root: Optional[int] = None):
        """j2t with ERR_HM served at every depth: entries[struct index] =
        (bytes, mask) the host wrote for that struct, None = the host failed
        (the ERR_HM code comes back). Returns (ret, out, field_cache) like
        j2t_hm2 (reference harness only)."""
        f = getattr(self.lib, self.p + "j2t_hm3")
        f.restype = C.c_uint64
        f.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_size_t, C.c_uint64, C.c_char_p, C.c_void_p,
                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t), C.c_void_p, C.c_size_t,
                      C.POINTER(C.c_size_t)]
        d = self._desc(flat.blob)
        root = flat.root_type if root is None else root
        ns = len(entries)
        off = (C.c_uint32 * max(ns, 1))()
        ln = (C.c_uint32 * max(ns, 1))()
        mk = (C.c_uint64 * max(ns, 1))()
        buf = b""
        for k, e in enumerate(entries):
            if e is None:
                ln[k] = 0xFFFFFFFF
                continue
            off[k], ln[k], mk[k] = len(buf), len(e[0]), e[1] & (2**64 - 1)
            buf += e[0]
        cap = 16 * len(json) + 64 * len(buf) + 65536
        out = C.create_string_buffer(cap)
        ol = C.c_size_t(0)
        fc = (C.c_int32 * 4096)()
        fl = C.c_size_t(0)
        ret = f(d, root, json, len(json), flags, buf + b"\0", off, ln, mk, out, cap, C.byref(ol), fc, 4096,
                C.byref(fl))
        if ret != 0 and (ret & 0xFF) != 21:
            return int(ret), b"", []
        return int(ret), out.raw[:ol.value], [int(fc[k]) for k in range(fl.value)]

    def set_hm_end_cb(self, fn):
        """A nested struct's ERR_HM_END served by `fn(struct_index, field_ids)
        -> bytes or None` (the test's host, handleUnmatchedFields + STOP);
        None = the host failed. fn None clears it (reference harness only)."""
        proto = C.CFUNCTYPE(C.c_long, C.c_uint32, C.POINTER(C.c_int32), C.c_size_t, C.POINTER(C.c_uint8), C.c_size_t)
        if fn is None:
            self._hm_end_keep = None
            self.lib.dgref_set_hm_end_cb(proto())
            return

        def tramp(si, ids, n, dst, cap):
            b = fn(int(si), [int(ids[k]) for k in range(n)])
            if b is None or len(b) > cap:
                return -1
            C.memmove(dst, bytes(b), len(b))
            return len(b)
        self._hm_end_keep = proto(tramp)
        self.lib.dgref_set_hm_end_cb(self._hm_end_keep)

    def j2t_batch(self, flat, msgs: Sequence[bytes], flags: int, nthreads: int = 1,
                  root: Optional[int] = None, slot_factor: int = 4, slot_pad: int = 64):
        """Batch API over an arena: returns (rets u64[n], outs list[bytes])."""
        arena, in_off = pack_arena(msgs)
        return self.j2t_arena(flat, arena, in_off, flags, nthreads, root, slot_factor, slot_pad)

    def j2t_arena(self, flat, arena: np.ndarray, in_off: np.ndarray, flags: int, nthreads: int = 1,
                  root: Optional[int] = None, slot_factor: int = 4, slot_pad: int = 64,
                  decode: bool = True):
        n = len(in_off) - 1
        lens = np.diff(in_off)
        out_off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(lens * slot_factor + slot_pad, out=out_off[1:])
        out = np.zeros(int(out_off[-1]) + 64, dtype=np.uint8)
        out_len = np.zeros(n, dtype=np.uint32)
        rets = np.zeros(n, dtype=np.uint64)
        d = self._desc(flat.blob)
        root = flat.root_type if root is None else root
        getattr(self.lib, self.p + "j2t_batch")(
            d, root, arena.ctypes.data, in_off.ctypes.data, n, flags, out.ctypes.data,
            out_off.ctypes.data, out_len.ctypes.data, rets.ctypes.data, nthreads)
        if not decode:
            return rets, (out, out_off, out_len)
        outs = []
        for i in range(n):
            if rets[i] != 0:
                outs.append(b"")
            elif int(out_len[i]) > int(out_off[i + 1] - out_off[i]):
                # the slot (len * slot_factor + slot_pad) was too small -- default
                # writes of a small message expand it (e.g. "{}" of a nested
                # struct with WRITE_DEFAULT: 120 bytes): the harness reported the
                # full length without the bytes; once more alone, with room
                a, b = int(in_off[i]), int(in_off[i + 1])
                r, o = self.j2t(flat, arena[a:b].tobytes(), flags, root)
                rets[i] = r
                outs.append(o)
            else:
                o = int(out_off[i])
                outs.append(out[o:o + int(out_len[i])].tobytes())
        return rets, outs


    def j2t_timed(self, flat, arena: np.ndarray, in_off: np.ndarray, flags: int, cpus: Sequence[int],
                  reps: int, root: Optional[int] = None, times: Optional[list] = None) -> float:
        """bench.py cpu_baseline: best-of-`reps` seconds for the whole arena
        (every pass's seconds appended to `times` when given),
        len(cpus) threads each pinned to one of `cpus` (byte-balanced shards,
        outputs preallocated here and first touched by an untimed pass).
        Reference harness only (oracle/_ref: dgref_j2t_timed)."""
        f = getattr(self.lib, self.p + "j2t_timed", None)
        if f is None:
            raise NotImplementedError("timed driver exists only in the reference harness")
        f.restype = C.c_int
        f.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p,
                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_int), C.c_int,
                      C.POINTER(C.c_double)]
        n = len(in_off) - 1
        in_off = np.ascontiguousarray(in_off, dtype=np.uint64)
        lens = np.diff(in_off)
        out_off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(lens * 4 + 64, out=out_off[1:])
        out = np.empty(int(out_off[-1]) + 64, dtype=np.uint8)
        out_len = np.zeros(n, dtype=np.uint32)
        rets = np.zeros(n, dtype=np.uint64)
        cpu_arr = (C.c_int * len(cpus))(*cpus)
        best = (C.c_double * (reps + 1))()
        root = flat.root_type if root is None else root
        rc = f(self._desc(flat.blob), root, arena.ctypes.data, in_off.ctypes.data, n, flags, out.ctypes.data,
               out_off.ctypes.data, out_len.ctypes.data, rets.ctypes.data, len(cpus), cpu_arr, reps, best)
        if rc != 0:
            raise RuntimeError("dgref_j2t_timed failed")
        if times is not None:
            times.extend(float(best[1 + r]) for r in range(reps))
        return float(best[0])


class RefT2J:
    """t2j checker: the C restatement of conv/t2j over the reference's own
    native encoders (oracle/ref_harness.c dgref_t2j)."""

    def __init__(self, lib: C.CDLL):
        self.lib = lib
        self.f = lib.dgref_t2j
        self.f.restype = C.c_uint64
        self.f.argtypes = [C.c_char_p, C.c_char_p, C.c_uint32, C.c_char_p, C.c_size_t, C.c_uint64,
                           C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]

    def t2j(self, flat, side: bytes, thrift: bytes, opts: int, root: Optional[int] = None) -> Tuple[int, bytes]:
        """(status, JSON): JSON b"" on error, except the exception's JSON
        with ConvertException (status 11)."""
        return self.t2j2(flat, side, thrift, opts, root)[:2]

    def t2j2(self, flat, side: bytes, thrift: bytes, opts: int, root: Optional[int] = None):
        """t2j plus the response-base span (DG_T2J_SKIP_RESP_BASE): (status,
        JSON, lo | hi << 32 or 2**64 - 1)."""
        f = self.lib.dgref_t2j2
        f.restype = C.c_uint64
        f.argtypes = [C.c_char_p, C.c_char_p, C.c_uint32, C.c_char_p, C.c_size_t, C.c_uint64,
                      C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t), C.POINTER(C.c_uint64)]
        root = flat.root_type if root is None else root
        cap = 8 * len(thrift) + 4096
        aux = C.c_uint64(0)
        for _ in range(2):
            out = C.create_string_buffer(cap)
            ol = C.c_size_t(0)
            ret = int(f(flat.blob, side, root, thrift, len(thrift), opts, out, cap, C.byref(ol), C.byref(aux)))
            if ret != 0 and (ret & 0xFF) != 11:
                return ret, b"", int(aux.value)
            if ol.value <= cap:
                return ret, out.raw[:ol.value], int(aux.value)
            cap = ol.value + 64
        raise RuntimeError("t2j oracle output did not fit")

    def t2j3(self, flat, side: bytes, thrift: bytes, opts: int, answers: bytes = b"", root: Optional[int] = None):
        """t2j2 with the host's writeHttpValue answers (DG_T2J_HM, one byte
        per call): (status, JSON or a stop's record, base span)."""
        f = self.lib.dgref_t2j3
        f.restype = C.c_uint64
        f.argtypes = [C.c_char_p, C.c_char_p, C.c_uint32, C.c_char_p, C.c_size_t, C.c_uint64,
                      C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t), C.POINTER(C.c_uint64), C.c_char_p,
                      C.c_uint32]
        root = flat.root_type if root is None else root
        cap = 8 * len(thrift) + 4096
        aux = C.c_uint64(0)
        for _ in range(2):
            out = C.create_string_buffer(cap)
            ol = C.c_size_t(0)
            ret = int(f(flat.blob, side, root, thrift, len(thrift), opts, out, cap, C.byref(ol), C.byref(aux),
                        bytes(answers), len(answers)))
            if ret != 0 and (ret & 0xFF) not in (11, 12):
                return ret, b"", int(aux.value)
            if ol.value <= cap:
                return ret, out.raw[:ol.value], int(aux.value)
            cap = ol.value + 64
        raise RuntimeError("t2j oracle output did not fit")


    def t2j_timed(self, flat, side: bytes, arena: np.ndarray, in_off: np.ndarray, opts: int, cpus: Sequence[int],
                  reps: int, root: Optional[int] = None, times: Optional[list] = None) -> float:
        """bench.py t2j cpu_baseline: best-of-`reps` seconds (each pass's to
        `times` when given) for the whole
        arena, len(cpus) threads pinned one per cpu (dgref_t2j_timed)."""
        f = self.lib.dgref_t2j_timed
        f.restype = C.c_int
        f.argtypes = [C.c_char_p, C.c_char_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64,
                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_int), C.c_int,
                      C.POINTER(C.c_double)]
        n = len(in_off) - 1
        in_off = np.ascontiguousarray(in_off, dtype=np.uint64)
        lens = np.diff(in_off)
        out_off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(lens * 8 + 256, out=out_off[1:])
        out = np.empty(int(out_off[-1]) + 64, dtype=np.uint8)
        out_len = np.zeros(n, dtype=np.uint32)
        rets = np.zeros(n, dtype=np.uint64)
        cpu_arr = (C.c_int * len(cpus))(*cpus)
        best = (C.c_double * (reps + 1))()
        root = flat.root_type if root is None else root
        rc = f(flat.blob, side, root, arena.ctypes.data, in_off.ctypes.data, n, opts, out.ctypes.data,
               out_off.ctypes.data, out_len.ctypes.data, rets.ctypes.data, len(cpus), cpu_arr, reps, best)
        if rc != 0:
            raise RuntimeError("dgref_t2j_timed failed")
        if times is not None:
            times.extend(float(best[1 + r]) for r in range(reps))
        return float(best[0])


def RefT2JOracle() -> Optional[RefT2J]:
    p = ref_lib_path()
    return RefT2J(C.CDLL(p)) if p else None


def physical_cpus() -> Tuple[List[int], int]:
    """CPUs this process may run on, one per physical core (lowest SMT
    sibling), and how many logical CPUs the affinity mask allows."""
    allowed = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    seen, pick = set(), []
    for c in allowed:
        try:
            base = "/sys/devices/system/cpu/cpu%d/topology/" % c
            with open(base + "physical_package_id") as fh:
                pkg = fh.read().strip()
            with open(base + "core_id") as fh:
                core = fh.read().strip()
            key = (pkg, core)
        except OSError:
            key = ("?", c)
        if key not in seen:
            seen.add(key)
            pick.append(c)
    return pick, len(allowed)


def pack_arena(msgs: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    lens = np.fromiter((len(m) for m in msgs), dtype=np.uint64, count=len(msgs))
    in_off = np.zeros(len(msgs) + 1, dtype=np.uint64)
    np.cumsum(lens, out=in_off[1:])
    arena = np.frombuffer(b"".join(msgs) + b"\0" * 64, dtype=np.uint8).copy()
    return arena, in_off


_ref_singleton = None
_port_singleton = None


def ref_lib_path() -> Optional[str]:
    cand = ["libdgref.so", "libdgref_sse.so"] if _cpu_has_avx2() else ["libdgref_sse.so"]
    for c in cand:
        p = os.path.join(HERE, "_ref", c)
        if os.path.exists(p):
            return p
    return None


def ref_utf8_validate(body: bytes) -> Optional[int]:
    """The reference's utf8_validate (native/utf8.c:183-212) on body: -1 if
    valid UTF-8, else the offset of the first invalid sequence; None when
    oracle/_ref was not built."""
    r = RefOracle()
    if r is None:
        return None
    f = r.lib.dgref_utf8_validate
    f.restype = C.c_long
    f.argtypes = [C.c_char_p, C.c_size_t]
    return int(f(body, len(body)))


def RefOracle() -> Optional[_Base]:
    """The reference's own C engine, or None if oracle/_ref was not built."""
    global _ref_singleton
    if _ref_singleton is None:
        p = ref_lib_path()
        if p is None:
            return None
        _ref_singleton = _Base(C.CDLL(p), "dgref_")
    return _ref_singleton


def PortOracle() -> _Base:
    """Our plain-C restatement (oracle/j2t_oracle.c)."""
    global _port_singleton
    if _port_singleton is None:
        p = os.path.join(HERE, "_build", "libj2t_oracle.so")
        if not os.path.exists(p):
            raise FileNotFoundError(f"{p} missing: run `make -C oracle oracle`")
        _port_singleton = _Base(C.CDLL(p), "dgo_")
    return _port_singleton


def unpack_ret(ret: int) -> Tuple[int, int, int]:
    """(code, pos, value) exactly as conv/j2t/impl_amd64.go:250-259 decode it."""
    code = ret & 0xFF
    pos = (ret >> 8) & 0xFFFFFFFF
    val = ret >> 40
    return code, pos, val
