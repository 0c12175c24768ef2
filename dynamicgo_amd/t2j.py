"""Host-side mirror of conv/t2j's API (Thrift binary -> JSON) over the HIP
kernels (dynamicgo_amd/csrc/t2j_device.h).

Reference surface (Go):
  t2j.NewBinaryConv(opts)              conv/t2j/conv.go:35
  (*BinaryConv).Do(ctx, desc, tbytes)  conv/t2j/conv.go:50-75
  (*BinaryConv).DoInto(...)            conv/t2j/conv.go:78-95
  the options it reads                 conv/api.go:52-121 (conv.Options)

Every call runs the HIP kernels in libdgj2t.so; there is no CPU fallback.
The Go-side options -- EnableHttpMapping (http.ResponseSetter callbacks),
EnableThriftBase (base.BaseResponse from the context) and ConvertException --
are not device features: they raise here, as the Go shim keeps them on the
host.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .conv import Context, Options, default_context
from .thrift import FlatDescriptor, flatten

# include/dgj2t_defs.h DG_T2J_*
T2J_BYTE_AS_UINT8 = 1 << 0
T2J_INT64_AS_STRING = 1 << 1
T2J_NULL_FOR_NAN_INF = 1 << 2
T2J_NO_BASE64 = 1 << 3
T2J_DISALLOW_UNKNOWN = 1 << 4
T2J_WRITE_DEFAULT = 1 << 5
T2J_WRITE_REQUIRE = 1 << 6
T2J_WRITE_OPTIONAL = 1 << 7
T2J_ENABLE_VM = 1 << 8

(E_READ, E_UNKNOWN_FIELD, E_DISMATCH_TYPE, E_UNSUPPORTED, E_NAN_INF, E_MISS_REQUIRED, E_NEEDS_HOST, E_DEPTH, E_WRITE,
 E_CONVERT) = range(1, 11)

# the meta.ErrCode behaviour the reference wraps each failure in
# (conv/t2j/impl.go: wrapError call sites; meta/error.go)
_BEHAVIOR = {E_READ: "ErrRead", E_UNKNOWN_FIELD: "ErrUnknownField", E_DISMATCH_TYPE: "ErrDismatchType",
             E_UNSUPPORTED: "ErrUnsupportedType", E_NAN_INF: "ErrWrite", E_MISS_REQUIRED: "ErrMissRequiredField",
             E_NEEDS_HOST: "ErrNotImplemented", E_DEPTH: "ErrStackOverflow",
             E_WRITE: "ErrWrite",       # truncated BYTE/I16/I32/I64/DOUBLE (conv/t2j/impl.go:200-236)
             E_CONVERT: "ErrConvert"}   # map key (buildinTypeToKey, conv/t2j/impl.go:355-358)
_READ_REASON = {1: "EOF", 2: "invalid data type", 3: "invalid data length", 4: "depth limit exceeded"}


def to_t2j_opts(o: Options) -> int:
    """The conv.Options fields conv/t2j/impl.go reads, as DG_T2J_* bits."""
    if o.EnableHttpMapping or o.EnableThriftBase or o.ConvertException:
        raise ValueError("EnableHttpMapping / EnableThriftBase / ConvertException are Go-side t2j features")
    f = 0
    if o.ByteAsUint8:
        f |= T2J_BYTE_AS_UINT8
    if o.Int642String:
        f |= T2J_INT64_AS_STRING
    if o.EncodeNullJSONForInfOrNan:
        f |= T2J_NULL_FOR_NAN_INF
    if o.NoBase64Binary:
        f |= T2J_NO_BASE64
    if o.DisallowUnknownField:
        f |= T2J_DISALLOW_UNKNOWN
    if o.WriteDefaultField:
        f |= T2J_WRITE_DEFAULT
    if o.WriteRequireField:
        f |= T2J_WRITE_REQUIRE
    if o.WriteOptionalField:
        f |= T2J_WRITE_OPTIONAL
    if o.EnableValueMapping:
        f |= T2J_ENABLE_VM
    return f


class T2JError(Exception):
    """A conversion error: the packed status word (code | pos << 8 | value <<
    40, pos = Thrift read offset) and the meta behaviour the reference
    reports for it."""

    def __init__(self, ret: int):
        self.ret = ret
        self.code, self.pos, self.value = ret & 0xFF, (ret >> 8) & 0xFFFFFFFF, ret >> 40
        self.behavior = _BEHAVIOR.get(self.code, "ErrConvert")
        super().__init__(f"[THRIFT2JSON] {self.behavior}: {self._detail()}")

    def _detail(self) -> str:
        c, v = self.code, self.value
        if c in (E_READ, E_WRITE):
            return f"{_READ_REASON.get(v, v)} at byte {self.pos}"
        if c == E_CONVERT:
            return (f"unsupported descriptor type {v & 0xFF} as MAP key" if v & 0x100 else
                    f"map key: {_READ_REASON.get(v, v)} at byte {self.pos}")
        if c == E_UNKNOWN_FIELD:
            return f"unknown field {v}"
        if c == E_DISMATCH_TYPE:
            return f"expect type {v >> 8} but got type {v & 0xFF}"
        if c == E_UNSUPPORTED:
            return f"unsupported type {v}"
        if c == E_NAN_INF:
            return "encounter Nan or Inf double"
        if c == E_MISS_REQUIRED:
            return f"required field {v} is not set"
        if c == E_DEPTH:
            return f"nesting beyond {v} containers"
        return f"code {c} value {v} at byte {self.pos}"


class BinaryConv:
    """t2j.BinaryConv (conv/t2j/conv.go:30-95) on the MI355X."""

    def __init__(self, opts: Optional[Options] = None, ctx: Optional[Context] = None):
        self.opts = opts or Options()
        self.ctx = ctx
        self._flat_cache = {}

    def set_options(self, opts: Options):
        self.opts = opts

    def _ctx(self) -> Context:
        if self.ctx is None:
            self.ctx = default_context()
        return self.ctx

    def _flat(self, desc) -> FlatDescriptor:
        if isinstance(desc, FlatDescriptor):
            return desc
        hit = self._flat_cache.get(id(desc))
        if hit is not None and hit[0] is desc:
            return hit[1]
        f = flatten(desc)
        self._flat_cache[id(desc)] = (desc, f)
        return f

    def do(self, desc, tbytes: bytes) -> Optional[bytes]:
        """Do: JSON bytes (None when empty, as the reference returns nil) or
        raises T2JError."""
        outs, rets = self.do_batch(desc, [tbytes])
        if rets[0] != 0:
            raise T2JError(int(rets[0]))
        return outs[0] if outs[0] else None

    def do_into(self, desc, tbytes: bytes, buf: bytearray):
        """DoInto: appends to buf."""
        out = self.do(desc, tbytes)
        if out:
            buf.extend(out)

    def do_batch(self, desc, msgs: Sequence[bytes]) -> Tuple[List[bytes], np.ndarray]:
        """Batch of independent Thrift messages -> (JSON outputs, statuses)."""
        opts = to_t2j_opts(self.opts)
        flat = self._flat(desc)
        ctx = self._ctx()
        n = len(msgs)
        lens = np.fromiter((len(m) for m in msgs), dtype=np.uint64, count=n)
        in_off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(lens, out=in_off[1:])
        arena = np.frombuffer(b"".join(msgs) + b"\0" * 16, dtype=np.uint8)
        rets = np.zeros(max(n, 1), dtype=np.uint64)
        out_off = np.zeros(n + 1, dtype=np.uint64)
        cap = int(lens.sum()) * 3 + 64 * n + 64
        out = np.zeros(cap, dtype=np.uint8)
        need = C.c_uint64(0)
        L = _lib.lib()
        d = ctx.desc_t2j(flat)
        rc = L.dg_t2j_batch_host(ctx.h, d, flat.root_type, arena.ctypes.data, in_off.ctypes.data, n, opts,
                                 out.ctypes.data, cap, out_off.ctypes.data, rets.ctypes.data, C.byref(need))
        if rc == -3 and need.value > cap:
            cap = int(need.value) + 64
            out = np.zeros(cap, dtype=np.uint8)
            rc = L.dg_t2j_batch_host(ctx.h, d, flat.root_type, arena.ctypes.data, in_off.ctypes.data, n, opts,
                                     out.ctypes.data, cap, out_off.ctypes.data, rets.ctypes.data, C.byref(need))
        _lib.check(rc)
        outs = [out[int(out_off[i]):int(out_off[i + 1])].tobytes() for i in range(n)]
        return outs, rets[:n]

    def do_device(self, desc, thrift, in_off, out, out_off, out_len, ret, stream=None):
        """Device-resident batch over torch tensors: thrift uint8[>= in_off[-1]
        + 16]; in_off/out_off int64[n+1] (8-aligned slots); out_len int32[n];
        ret int64[n]. Asynchronous on `stream` (default: torch's current
        stream). Statuses DG_ST_OUT_OVERFLOW (0xF0) leave out_len = the bytes
        the message needs."""
        opts = to_t2j_opts(self.opts)
        flat = self._flat(desc)
        ctx = self._ctx()
        n = in_off.numel() - 1
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(thrift.device)
        _lib.check(_lib.lib().dg_t2j_batch_device(
            ctx.h, ctx.desc_t2j(flat), flat.root_type, thrift.data_ptr(), in_off.data_ptr(), n, opts,
            out.data_ptr(), out_off.data_ptr(), out_len.data_ptr(), ret.data_ptr(), stream.cuda_stream))


def new_binary_conv(opts: Optional[Options] = None) -> BinaryConv:
    """t2j.NewBinaryConv (conv/t2j/conv.go:35)."""
    return BinaryConv(opts)
