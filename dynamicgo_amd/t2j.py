"""Host-side mirror of conv/t2j's API (Thrift binary -> JSON) over the HIP
kernels (dynamicgo_amd/csrc/t2j_device.h).

Reference surface (Go):
  t2j.NewBinaryConv(opts)              conv/t2j/conv.go:35
  (*BinaryConv).Do(ctx, desc, tbytes)  conv/t2j/conv.go:50-75
  (*BinaryConv).DoInto(...)            conv/t2j/conv.go:78-95
  the options it reads                 conv/api.go:52-121 (conv.Options)

Every call runs the HIP kernels in libdgj2t.so; there is no CPU fallback.
The Go-side options are split between the device and this host part:
  * ConvertException (conv/t2j/impl.go:154-187): the device stops at the root's
    exception field and keeps its JSON (DG_T2J_E_EXCEPTION); here it becomes
    the error, errors.New(json), as Do returns it;
  * EnableThriftBase with a context BaseResp (readResponseBase,
    impl.go:54-72): the device skips the root's response-base field and
    reports its span; here the BaseResp is FastRead from those bytes;
  * EnableHttpMapping (writeHttpValue, impl.go:515-588): the mapped fields'
    values go to the http.ResponseSetter, see do_batch.
"""
from __future__ import annotations

import ctypes as C
import struct as _st
from typing import Dict, List, Optional, Sequence, Tuple

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
T2J_CONVERT_EXC = 1 << 9
T2J_SKIP_RESP_BASE = 1 << 10

(E_READ, E_UNKNOWN_FIELD, E_DISMATCH_TYPE, E_UNSUPPORTED, E_NAN_INF, E_MISS_REQUIRED, E_NEEDS_HOST, E_DEPTH, E_WRITE,
 E_CONVERT, E_EXCEPTION) = range(1, 12)

# the meta.ErrCode behaviour the reference wraps each failure in
# (conv/t2j/impl.go: wrapError call sites; meta/error.go)
_BEHAVIOR = {E_READ: "ErrRead", E_UNKNOWN_FIELD: "ErrUnknownField", E_DISMATCH_TYPE: "ErrDismatchType",
             E_UNSUPPORTED: "ErrUnsupportedType", E_NAN_INF: "ErrWrite", E_MISS_REQUIRED: "ErrMissRequiredField",
             E_NEEDS_HOST: "ErrNotImplemented", E_DEPTH: "ErrStackOverflow",
             E_WRITE: "ErrWrite",       # truncated BYTE/I16/I32/I64/DOUBLE (conv/t2j/impl.go:200-236)
             E_CONVERT: "ErrConvert"}   # map key (buildinTypeToKey, conv/t2j/impl.go:355-358)
_READ_REASON = {1: "EOF", 2: "invalid data type", 3: "invalid data length", 4: "depth limit exceeded"}


def to_t2j_opts(o: Options, base: bool = False) -> int:
    """The conv.Options fields conv/t2j/impl.go reads, as DG_T2J_* bits;
    base: a BaseResp is in the context (EnableThriftBase skips the field)."""
    if o.EnableHttpMapping:
        raise ValueError("EnableHttpMapping: use BinaryConv.do_batch_http (the ResponseSetter callbacks)")
    f = 0
    if o.ConvertException:
        f |= T2J_CONVERT_EXC
    if o.EnableThriftBase and base:
        f |= T2J_SKIP_RESP_BASE
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


class T2JException(Exception):
    """ConvertException (conv/t2j/impl.go:183-185): the message held an
    exception field; the error's text is that field's JSON, errors.New(json)."""

    def __init__(self, js: bytes):
        super().__init__(js.decode("utf-8", "replace"))
        self.json = js


class ThriftReadError(ValueError):
    pass


def _skip(b: bytes, p: int, t: int, depth: int = 64) -> int:
    """skipType on Thrift binary (thrift/binary_skip.go), host side: the
    position after the value of wire type t at p."""
    fs = {2: 1, 3: 1, 6: 2, 8: 4, 4: 8, 10: 8}.get(t)
    if fs:
        if p + fs > len(b):
            raise ThriftReadError("EOF")
        return p + fs
    if depth <= 0:
        raise ThriftReadError("depth limit exceeded")
    if t == 11:
        if p + 4 > len(b):
            raise ThriftReadError("EOF")
        n = _st.unpack_from(">I", b, p)[0]
        if p + 4 + n > len(b):
            raise ThriftReadError("EOF")
        return p + 4 + n
    if t == 12:
        while True:
            if p >= len(b):
                raise ThriftReadError("EOF")
            ft = b[p]
            p += 1
            if ft == 0:
                return p
            p = _skip(b, p + 2, ft, depth - 1)
    if t == 13:
        if p + 6 > len(b):
            raise ThriftReadError("EOF")
        kt, vt, n = b[p], b[p + 1], _st.unpack_from(">i", b, p + 2)[0]
        p += 6
        for _ in range(max(n, 0)):
            p = _skip(b, _skip(b, p, kt, depth - 1), vt, depth - 1)
        return p
    if t in (14, 15):
        if p + 5 > len(b):
            raise ThriftReadError("EOF")
        et, n = b[p], _st.unpack_from(">i", b, p + 1)[0]
        p += 5
        for _ in range(max(n, 0)):
            p = _skip(b, p, et, depth - 1)
        return p
    raise ThriftReadError("invalid data type %d" % t)


class BaseResp:
    """base.BaseResp (testdata/idl/base.thrift:19-23: 1: string StatusMessage
    = "", 2: i32 StatusCode = 0, 3: optional map<string, string> Extra), the
    context object EnableThriftBase fills (conv.CtxKeyThriftRespBase)."""

    def __init__(self, StatusMessage: str = "", StatusCode: int = 0, Extra: Optional[Dict[str, str]] = None):
        self.StatusMessage, self.StatusCode, self.Extra = StatusMessage, StatusCode, Extra

    def __eq__(self, o):
        return isinstance(o, BaseResp) and (self.StatusMessage, self.StatusCode, self.Extra) == \
            (o.StatusMessage, o.StatusCode, o.Extra)

    def __repr__(self):
        return "BaseResp(%r, %r, %r)" % (self.StatusMessage, self.StatusCode, self.Extra)

    def fast_read(self, b: bytes):
        """The kitex FastRead: fields by id and wire type, others skipped."""
        p = 0

        def rstr(p):
            if p + 4 > len(b):
                raise ThriftReadError("EOF")
            n = _st.unpack_from(">I", b, p)[0]
            if p + 4 + n > len(b):
                raise ThriftReadError("EOF")
            return b[p + 4:p + 4 + n].decode("utf-8", "surrogateescape"), p + 4 + n
        while True:
            if p >= len(b):
                raise ThriftReadError("EOF")
            t = b[p]
            if t == 0:
                return p + 1
            if p + 3 > len(b):
                raise ThriftReadError("EOF")
            fid = _st.unpack_from(">h", b, p + 1)[0]
            p += 3
            if fid == 1 and t == 11:
                self.StatusMessage, p = rstr(p)
            elif fid == 2 and t == 8:
                if p + 4 > len(b):
                    raise ThriftReadError("EOF")
                self.StatusCode = _st.unpack_from(">i", b, p)[0]
                p += 4
            elif fid == 3 and t == 13 and p + 6 <= len(b) and b[p] == 11 and b[p + 1] == 11:
                n = _st.unpack_from(">i", b, p + 2)[0]
                p += 6
                m = {}
                for _ in range(max(n, 0)):
                    k, p = rstr(p)
                    v, p = rstr(p)
                    m[k] = v
                self.Extra = m
            else:
                p = _skip(b, p, t)


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

    def do(self, desc, tbytes: bytes, resp=None, base: Optional[BaseResp] = None) -> Optional[bytes]:
        """Do: JSON bytes (None when empty, as the reference returns nil) or
        raises T2JError / T2JException (ConvertException) / ThriftReadError
        (the context BaseResp did not read). resp: the context's
        http.ResponseSetter (EnableHttpMapping); base: its BaseResp, filled
        in place (EnableThriftBase)."""
        outs, errs = self.do_batch_errors(desc, [tbytes], [resp], [base])
        if errs[0] is not None:
            raise errs[0]
        return outs[0] if outs[0] else None

    def do_into(self, desc, tbytes: bytes, buf: bytearray, resp=None, base: Optional[BaseResp] = None):
        """DoInto: appends to buf (also the exception's JSON before raising
        T2JException, as the reference leaves it in the buffer)."""
        try:
            out = self.do(desc, tbytes, resp, base)
        except T2JException as e:
            buf.extend(e.json)
            raise
        if out:
            buf.extend(out)

    def do_batch_errors(self, desc, msgs: Sequence[bytes], resps=None, bases=None):
        """Do over a batch with the context's objects per message: (outputs,
        errors) with errors[i] None, T2JError, T2JException or
        ThriftReadError."""
        n = len(msgs)
        bases = list(bases) if bases is not None else [None] * n
        outs, rets, aux = self._batch(desc, msgs, with_base=any(b is not None for b in bases))
        errs: List[Optional[Exception]] = [None] * n
        for i in range(n):
            r = int(rets[i])
            if (r & 0xFF) == E_EXCEPTION:
                errs[i], outs[i] = T2JException(outs[i]), b""
                continue
            if r != 0:
                errs[i] = T2JError(r)
                continue
            if bases[i] is not None and aux is not None and int(aux[i]) != 2**64 - 1:
                lo, hi = int(aux[i]) & 0xFFFFFFFF, int(aux[i]) >> 32
                try:
                    bases[i].fast_read(bytes(msgs[i][lo:hi]))  # readResponseBase's FastRead
                except ThriftReadError as e:
                    errs[i], outs[i] = e, b""
        return outs, errs

    def do_batch(self, desc, msgs: Sequence[bytes]) -> Tuple[List[bytes], np.ndarray]:
        """Batch of independent Thrift messages -> (JSON outputs, statuses)."""
        outs, rets, _ = self._batch(desc, msgs)
        return outs, rets

    def _batch(self, desc, msgs: Sequence[bytes], with_base: bool = False):
        opts = to_t2j_opts(self.opts, with_base)
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
        aux = np.zeros(max(n, 1), dtype=np.uint64) if opts & T2J_SKIP_RESP_BASE else None
        for _ in range(2):
            rc = L.dg_t2j_batch_host_aux(ctx.h, d, flat.root_type, arena.ctypes.data, in_off.ctypes.data, n, opts,
                                         out.ctypes.data, cap, out_off.ctypes.data, rets.ctypes.data,
                                         C.byref(need), aux.ctypes.data if aux is not None else None)
            if rc == -3 and need.value > cap:
                cap = int(need.value) + 64
                out = np.zeros(cap, dtype=np.uint8)
                continue
            break
        _lib.check(rc)
        outs = [out[int(out_off[i]):int(out_off[i + 1])].tobytes() for i in range(n)]
        return outs, rets[:n], aux

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
