"""Host-side mirror of conv/j2t's API over the HIP transcoder.

Reference surface (Go):
  conv.Options                      conv/api.go:52-121
  j2t.NewBinaryConv(opts)           conv/j2t/conv.go:36
  (*BinaryConv).Do(ctx, desc, json) conv/j2t/conv.go:53-77
  (*BinaryConv).DoInto(...)         conv/j2t/conv.go:81-96
  toFlags(opts)                     conv/j2t/conv.go:98-127
  explainNativeError(ret, in)       conv/j2t/impl_amd64.go:261-298

Additions for the batched device path: ``BinaryConv.do_batch`` (host arenas)
and ``BinaryConv.do_device`` (arenas already resident in HBM, torch tensors).
Every call runs the HIP kernels in libdgj2t.so; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import struct as _st
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from . import http as H
from .thrift import FlatDescriptor, TypeDescriptor, flatten, TYPE_NAMES, ValueMappingError

# flag bits (native/thrift.h:23-32, internal/types/types.go:81-92)
F_ALLOW_UNKNOWN = 1
F_WRITE_DEFAULT = 1 << 1
F_VALUE_MAPPING = 1 << 2
F_HTTP_MAPPING = 1 << 3
F_STRING_INT = 1 << 4
F_WRITE_REQUIRE = 1 << 5
F_NO_BASE64 = 1 << 6
F_WRITE_OPTIONAL = 1 << 7
F_TRACE_BACK = 1 << 8
F_NO_WRITE_BASE = 1 << 9
F_VALIDATE_UTF8 = 1 << 16  # extension, off by default
F_FLAT_PATH = 1 << 19      # extension: force the field-major flat kernel (default for flat roots, messages <= 256 B)
F_HM_SPLIT = 1 << 20       # extension: root HTTP mappings written by the host (do_batch_hm_split)
F_NO_FLAT_PATH = 1 << 21   # extension: the lane-per-message small kernel even for a flat root (testing)

DG_ST_OUT_OVERFLOW = 0xF0
DG_ST_DEEP = 0xF1
DG_ST_HM_END = 0xF2
DG_ST_HM_ERR = 0xF3
DG_ST_HM_END_AT = 0xF4
DG_ST_CB_LIST = 0xF5  # DG_F_CB_COLLECT: every callback of one pass recorded (dgj2t_defs.h)
E_VM_END = 24  # ERR_VM_END (native/native.h:70): a non-inline value mapping for the host
F_CB_COLLECT = 1 << 22  # extension: record the callbacks of a pass and convert on (2 passes for k callbacks)
_CB_CODES = (E_VM_END, DG_ST_HM_END_AT, DG_ST_CB_LIST)


def _cb_records(rec: bytes, r: int):
    """The callbacks a message stopped at, [(status, record)] in message
    order: a DG_ST_CB_LIST slot holds every one of the pass (each behind the
    status word its stop would have returned), the others one."""
    if (r & 0xFF) != DG_ST_CB_LIST:
        return [(r, rec)]
    out, at = [], 0
    for _ in range(r >> 40):
        st = int.from_bytes(rec[at:at + 8], "big")
        at += 8
        n = 16 if (st & 0xFF) == E_VM_END else 8 + 8 * (st >> 40)
        out.append((st, rec[at:at + n]))
        at += n
    return out

# internal/types/types.go:107-131 ParsingError messages
_ERR_MSG = {0: "ok", 1: "eof", 2: "invalid char", 3: "invalid escape char", 4: "invalid unicode escape",
            5: "integer overflow", 6: "invalid number format", 7: "recursion exceeded max depth",
            8: "float number is infinity", 9: "dismatched type", 10: "required field is not set",
            11: "unsupported type", 12: "unknown field", 13: "dismatched types", 14: "decode base64 error",
            16: "out of memory of bitmap", 17: "out of memory of buffer", 18: "out of memory of key",
            19: "http-mapping", 20: "unsupported value-mapping", 21: "http-mapping end",
            22: "out of memory of field", 23: "out of memory of field value", 24: "value-mapping end"}
_J2T_STATES = {0: "J2T_VAL", 1: "J2T_ARR", 2: "J2T_OBJ", 3: "J2T_KEY", 4: "J2T_ELEM", 5: "J2T_ARR_0",
               6: "J2T_OBJ_0", 16: "J2T_VM"}


@dataclass
class Options:
    """conv.Options (conv/api.go:52-121), the fields j2t reads."""
    EnableValueMapping: bool = False
    EnableHttpMapping: bool = False
    EnableThriftBase: bool = False
    String2Int64: bool = False
    NoBase64Binary: bool = False
    WriteOptionalField: bool = False
    WriteDefaultField: bool = False
    WriteRequireField: bool = False
    DisallowUnknownField: bool = False
    ReadHttpValueFallback: bool = False
    TracebackRequredOrRootFields: bool = False
    MergeBaseFunc: Optional[object] = None  # func(json_base, ctx_base) -> Base (conv/api.go:118-120)
    ValidateUTF8: bool = False  # extension (north_star: "UTF-8 validation"), default off
    # fields only the reverse path (t2j, dynamicgo_amd.t2j) reads
    Int642String: bool = False
    ByteAsUint8: bool = False
    EncodeNullJSONForInfOrNan: bool = False
    ConvertException: bool = False
    WriteHttpValueFallback: bool = False
    OmitHttpMappingErrors: bool = False
    UseKitexHttpEncoding: bool = False


def to_flags(o: Options) -> int:
    """toFlags conv/j2t/conv.go:98-127."""
    f = 0
    if o.WriteDefaultField:
        f |= F_WRITE_DEFAULT
    if not o.DisallowUnknownField:
        f |= F_ALLOW_UNKNOWN
    if o.EnableValueMapping:
        f |= F_VALUE_MAPPING
    if o.EnableHttpMapping:
        f |= F_HTTP_MAPPING
    if o.String2Int64:
        f |= F_STRING_INT
    if o.WriteRequireField:
        f |= F_WRITE_REQUIRE
    if o.NoBase64Binary:
        f |= F_NO_BASE64
    if o.WriteOptionalField:
        f |= F_WRITE_OPTIONAL
    if o.ReadHttpValueFallback:
        f |= F_TRACE_BACK
    if o.ValidateUTF8:
        f |= F_VALIDATE_UTF8
    return f


def unpack_ret(ret: int) -> Tuple[int, int, int]:
    """(code, pos, value): getErrCode/getPos/getValue conv/j2t/impl_amd64.go:250-259."""
    return ret & 0xFF, (ret >> 8) & 0xFFFFFFFF, ret >> 40


# meta.ErrorCode behaviours explainNativeError files each native code under
# (conv/j2t/impl_amd64.go:261-298, meta/error.go)
_BEHAVIOR = {2: "ErrRead", 6: "ErrConvert", 11: "ErrUnsupportedType", 20: "ErrUnsupportedType",
             9: "ErrDismatchType", 10: "ErrMissRequiredField", 12: "ErrUnknownField", 7: "ErrStackOverflow",
             14: "ErrRead"}


class J2TError(Exception):
    """A conversion error, carrying the reference's packed status word and the
    meta behaviour explainNativeError assigns it (default ErrConvert)."""

    def __init__(self, ret: int, msg: str):
        super().__init__(msg)
        self.ret = ret
        self.code, self.pos, self.value = unpack_ret(ret)
        self.behavior = _BEHAVIOR.get(self.code, "ErrConvert")


def _locate(src: bytes, ip: int) -> str:
    # json.SyntaxError.Locate: a window around the position
    lo, hi = max(0, ip - 10), min(len(src), ip + 10)
    return "\n\n\t%s\n\n\t%s^%s\n" % (src[lo:hi].decode("utf-8", "replace"), "." * (ip - lo), "." * (hi - ip))


def explain_native_error(ret: int, src: bytes) -> str:
    """explainNativeError conv/j2t/impl_amd64.go:261-298 (message text)."""
    e, ip, v = unpack_ret(ret)
    loc = _locate(src, ip)
    if e == 2:
        ch, st = v >> 8, v & 0xFF
        return "invalid char '%s' for state %s, near %d of %s" % (chr(ch & 0xFF), _J2T_STATES.get(st, st), ip, loc)
    if e == 6:
        return "unexpected number type %d, near %d of %s" % (v, ip, loc)
    if e == 11:
        return "unsupported thrift type %s, near %d of %s" % (TYPE_NAMES.get(v, v), ip, loc)
    if e == 20:
        return "unsupported value-mapping type %d, near %d of %r" % (v, ip, loc)
    if e == 9:
        return "expect type %s but got type %d, near %d of %s" % (TYPE_NAMES.get(v >> 8, v >> 8), v & 0xFF, ip, loc)
    if e == 10:
        return "missing required field %d, near %d of %s" % (v, ip, loc)
    if e == 12:
        n = max(ip - v - 1, 0)
        return "unknown field '%s', near %d of %s" % (src[n:ip - 1].decode("utf-8", "replace"), ip, loc)
    if e == 7:
        return "stack %d overflow, near %d of %s" % (v, ip, loc)
    if e == 14:
        return "decode base64 error: illegal base64 data at input byte %d, near %d of %s" % (v, ip, loc)
    return "native error %r, value %d, near %d of %s" % (_ERR_MSG.get(e, "unknown"), v, ip, loc)


class Context:
    """One HIP device: stream + workspaces (dg_ctx)."""

    def __init__(self, device: int = 0):
        L = _lib.lib()
        h = C.c_void_p()
        _lib.check(L.dg_ctx_create(device, C.byref(h)))
        self.h = h
        self.device = device
        self._descs = {}
        self._t2j = set()

    def desc_t2j(self, flat: FlatDescriptor):
        """desc() with the t2j side table attached (dg_desc_attach_t2j)."""
        d = self.desc(flat)
        if flat.blob not in self._t2j:
            from .thrift import flatten_t2j
            side = flatten_t2j(flat)
            _lib.check(_lib.lib().dg_desc_attach_t2j(d, side, len(side)))
            self._t2j.add(flat.blob)
        return d

    def desc(self, flat: FlatDescriptor):
        """Device-resident copy of a flattened descriptor (cached by content)."""
        d = self._descs.get(flat.blob)
        if d is None:
            h = C.c_void_p()
            _lib.check(_lib.lib().dg_desc_create(self.h, flat.blob, len(flat.blob), C.byref(h)))
            d = h
            self._descs[flat.blob] = d
        return d

    def stats(self, reset: bool = False):
        """(bails, deeps): messages the fast path handed to the exact machine
        and messages redone with the deep stack, since the last reset."""
        b, d = C.c_uint64(0), C.c_uint64(0)
        _lib.check(_lib.lib().dg_ctx_stats(self.h, C.byref(b), C.byref(d), int(reset)))
        return int(b.value), int(d.value)

    def set_knob(self, name: str, value: int):
        """A routing knob (dg_ctx_set_knob, include/dgj2t.h): "flat",
        "wave_min", "wave_occ", "small_mpw", "list_blocks", "t2j_spread",
        "t2j_wave_min", "flat_wrap"."""
        _lib.check(_lib.lib().dg_ctx_set_knob(self.h, name.encode(), int(value)))

    def get_knob(self, name: str) -> int:
        v = C.c_int64(0)
        _lib.check(_lib.lib().dg_ctx_get_knob(self.h, name.encode(), C.byref(v)))
        return int(v.value)

    def knobs(self, **kv):
        """Context manager: set knobs, restore them on exit."""
        import contextlib

        @contextlib.contextmanager
        def cm():
            old = {k: self.get_knob(k) for k in kv}
            try:
                for k, v in kv.items():
                    self.set_knob(k, v)
                yield self
            finally:
                for k, v in old.items():
                    self.set_knob(k, v)
        return cm()

    def close(self):
        L = _lib.lib()
        for d in self._descs.values():
            L.dg_desc_destroy(d)
        self._descs.clear()
        self._t2j.clear()
        if self.h:
            L.dg_ctx_destroy(self.h)
            self.h = None


_default_ctx: Optional[Context] = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


class BinaryConv:
    """j2t.BinaryConv (conv/j2t/conv.go:31-96) on the MI355X."""

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
        # keyed by id() but holding the descriptor itself: a live entry pins
        # its object, so the id cannot be reused by another descriptor (the
        # reference caches by *TypeDescriptor pointer the same way)
        hit = self._flat_cache.get(id(desc))
        if hit is not None and hit[0] is desc:
            return hit[1]
        f = flatten(desc)
        self._flat_cache[id(desc)] = (desc, f)
        return f

    def _check_opts(self):
        """EnableHttpMapping is accepted: the GPU returns the reference's
        callback codes (ERR_HM at a struct with HTTP-mapped fields,
        native/thrift.c:1119-1123; ERR_HM_END, native/thrift.c:898-903), which
        the Go host serves from the request (conv/j2t/impl_amd64.go:174-198);
        structs without mapped fields convert as usual."""

    def do(self, desc, jbytes: bytes, req: Optional["H.HTTPRequest"] = None,
           base: Optional["H.Base"] = None) -> Optional[bytes]:
        """Do (conv/j2t/conv.go:53-77): returns Thrift bytes (None for an empty
        result) or raises J2TError / http.ConvError. `req` is the context's
        conv.CtxKeyHTTPRequest (EnableHttpMapping), `base` its
        conv.CtxKeyThriftReqBase (EnableThriftBase)."""
        if req is not None or base is not None:
            outs, errs = self.do_batch_http(desc, [jbytes], [req], [base])
            if errs[0] is not None:
                raise errs[0]
            return outs[0] or None
        outs, errs = self.do_batch_errors(desc, [jbytes])
        if errs[0] is not None:
            raise errs[0]
        return outs[0] if outs[0] else None

    def do_into(self, desc, jbytes: bytes, buf: bytearray, req=None, base=None):
        """DoInto: appends to buf."""
        out = self.do(desc, jbytes, req, base)
        if out:
            buf.extend(out)

    def _td(self, desc) -> TypeDescriptor:
        if isinstance(desc, FlatDescriptor):
            raise TypeError("the HTTP-mapping path needs the TypeDescriptor (its annotations), not a flat blob")
        return desc

    def _nested(self, flags: int):
        """writeStringValue's doImpl recursion (conv/j2t/impl.go:140-145): a
        JSON-encoded complex value converted as its field's type, top=false,
        on the GPU."""
        def conv_nested(f, val: str) -> bytes:
            src = val.encode("utf-8", "surrogateescape")
            outs, rets = self.do_batch(f.type, [src], extra_flags=flags & ~to_flags(self.opts))
            if int(rets[0]) != 0:
                raise H.ConvError("ErrConvert", "failed to convert value of field '%s'" % f.name,
                                  J2TError(int(rets[0]), explain_native_error(int(rets[0]), src)))
            return outs[0]
        return conv_nested

    def _host_cb(self, flat: FlatDescriptor, msgs: Sequence[bytes], flags: int, hm_rows=None, n_hm: int = 0,
                 hm_bytes: bytes = b"", vm_answers=None):
        """dg_j2t_batch_host_cb over `msgs` with the host's callback answers:
        hm_rows[k] = message k's n_hm (off, len, mask) HTTP-mapping entries
        into hm_bytes, vm_answers[k] = the Thrift bytes of its first
        value-mapping answers (dgj2t_defs.h dg_cb_tables). Returns
        (outputs, packed statuses); an output holds the partial output and
        requires words for DG_ST_HM_END, the 16-byte record for ERR_VM_END."""
        ctx = self._ctx()
        L = _lib.lib()
        if flags & (F_VALUE_MAPPING | F_HM_SPLIT):
            flags |= F_CB_COLLECT  # every callback of a pass at once (k callbacks: 2 passes)
        m = len(msgs)
        lens = np.fromiter((len(x) for x in msgs), dtype=np.uint64, count=m)
        in_off = np.zeros(m + 1, dtype=np.uint64)
        np.cumsum(lens, out=in_off[1:])
        arena = np.frombuffer(b"".join(msgs) + b"\0" * 16, dtype=np.uint8)
        pool = bytearray(hm_bytes)
        cb = None
        keep = []
        extra = 0  # output the host's answers add per message (first capacity)
        if hm_rows is not None or vm_answers is not None:
            cb = _lib.CBTables()
            if hm_rows is not None and n_hm:
                tab = (_lib.HMEntry * (m * n_hm))()
                for k, row in enumerate(hm_rows):
                    for j, (off, ln, mask) in enumerate(row):
                        tab[k * n_hm + j] = _lib.HMEntry(off, ln, mask & (2**64 - 1))
                cb.hm_tab, cb.n_hm = C.cast(tab, C.c_void_p), n_hm
                keep.append(tab)
            if vm_answers is not None:
                vt = (_lib.VMEntry * max(m, 1))()
                for k, ans in enumerate(vm_answers):
                    vt[k] = _lib.VMEntry(len(pool), len(ans))
                    for a in ans:
                        pool += len(a).to_bytes(4, "little") + a
                cb.ans_tab = C.cast(vt, C.c_void_p)
                keep.append(vt)
            pb = (C.c_uint8 * (len(pool) + 8)).from_buffer_copy(bytes(pool) + b"\0" * 8)
            keep.append(pb)
            cb.bytes, cb.len = C.cast(pb, C.c_void_p), len(pool)
            extra = len(pool) + 64 * m
        rets = np.zeros(max(m, 1), dtype=np.uint64)
        out_off = np.zeros(m + 1, dtype=np.uint64)
        cap = int(lens.sum()) * 4 + 64 * m + 64 + extra
        need = C.c_uint64(0)
        for _ in range(2):
            out = np.zeros(cap, dtype=np.uint8)
            rc = L.dg_j2t_batch_host_cb(ctx.h, ctx.desc(flat), flat.root_type, arena.ctypes.data, in_off.ctypes.data,
                                        m, flags, C.byref(cb) if cb is not None else None, out.ctypes.data, cap,
                                        out_off.ctypes.data, rets.ctypes.data, C.byref(need))
            if rc == -3 and need.value > cap:  # DG_E_NOMEM: once more with the size it needs
                cap = int(need.value) + 64
                continue
            break
        _lib.check(rc)
        return [out[int(out_off[k]):int(out_off[k + 1])].tobytes() for k in range(m)], rets[:m]

    def _serve_callbacks(self, flat: FlatDescriptor, msgs: Sequence[bytes], flags: int, outs, rets, errs,
                         hm_rows=None, n_hm: int = 0, hm_bytes: bytes = b"", hm_end=None):
        """The reference's mid-message Go callbacks (handleError,
        conv/j2t/impl_amd64.go:169-247), served and resumed: each message the
        device stopped at a callback gets the host's answer appended to its
        answers (dg_cb_entry) and is converted again, until it finishes.
          * ERR_VM_END (native/thrift.c:641-665) -> handleValueMapping
            (impl_amd64.go:117-155): the field header, then the field's
            ValueMapping.write on the value's JSON text;
          * DG_ST_HM_END_AT, a nested struct's ERR_HM_END -> hm_end(i, struct,
            field ids): handleUnmatchedFields' bytes (impl_amd64.go:71-115).
        In place on outs / rets / errs; a failing callback leaves the message
        its stop status and its error in errs."""
        answers = {}

        def serve(i, r, rec):  # one callback -> its answer bytes, or raise
            src = msgs[i]
            if (r & 0xFF) == DG_ST_HM_END_AT:
                si = _st.unpack(">Q", rec[:8])[0]
                sd = flat.structs[si]
                order = sorted(sd.fields, key=lambda f: f.id)
                ids = []
                for w in range(r >> 40):
                    bits = _st.unpack(">Q", rec[8 + 8 * w:16 + 8 * w])[0]
                    ids += [order[64 * w + b].id for b in range(64) if (bits >> b) & 1 and 64 * w + b < len(order)]
                if hm_end is None:
                    raise H.ConvError("ErrInvalidParam", "http request is nil")
                return hm_end(i, sd, ids)
            end = r >> 8
            start, fidx = _st.unpack(">QQ", rec[:16])
            f = flat.fields[fidx] if fidx < len(getattr(flat, "fields", [])) else None
            if f is None:
                raise H.ConvError("ErrConvert", "unknown field id for value-mapping")
            if end >= len(src) or start > end:  # impl_amd64.go:132-134
                raise H.ConvError("ErrConvert", "invalid value-mapping position")
            try:
                if f.value_mapping is None:
                    raise ValueMappingError("no value mapping registered for type %d" % f.vm)
                val = f.value_mapping.write(f, bytes(src[start:end]))
            except Exception as e:  # any Write error (impl_amd64.go:137-139)
                raise H.ConvError("ErrConvert", "failed to convert field '%s' value" % f.name, e)
            return bytes([f.type.type]) + _st.pack(">h", f.id) + bytes(val)

        todo = [i for i in range(len(msgs)) if (int(rets[i]) & 0xFF) in _CB_CODES and errs[i] is None]
        while todo:
            live = []
            for i in todo:
                rec, r = outs[i], int(rets[i])
                outs[i] = b""
                try:
                    recs = _cb_records(rec, r)
                    if not recs:  # an empty record list would rerun the message unchanged forever
                        raise H.ConvError("ErrConvert", "callback record list is empty")
                    # served in the order the message meets them: a failing
                    # callback is the error, as in the reference's Go loop
                    for rk, reck in recs:
                        answers.setdefault(i, []).append(serve(i, rk, reck))
                except H.ConvError as e:
                    errs[i] = e
                    continue
                live.append(i)
            if not live:
                break
            o2, r2 = self._host_cb(flat, [msgs[i] for i in live], flags,
                                   [hm_rows[i] for i in live] if hm_rows is not None else None, n_hm, hm_bytes,
                                   [answers[i] for i in live])
            for k, i in enumerate(live):
                outs[i], rets[i] = o2[k], r2[k]
            todo = [i for i in live if (int(rets[i]) & 0xFF) in _CB_CODES]

    def do_batch_errors(self, desc, msgs: Sequence[bytes], extra_flags: int = 0):
        """BinaryConv.Do over a batch (conv/j2t/conv.go:53-77): (outputs,
        errors), errors[i] None, a J2TError (the native status) or an
        http.ConvError (a value-mapping callback that failed)."""
        outs, rets, vm_errs = self._do_batch(desc, msgs, extra_flags)
        errs = [None] * len(msgs)
        for i, r in enumerate(rets):
            if i in vm_errs:
                errs[i] = vm_errs[i]
            elif int(r) != 0:
                errs[i] = J2TError(int(r), explain_native_error(int(r), msgs[i]))
        return outs, errs

    def do_batch_http(self, desc, msgs: Sequence[bytes], reqs: Sequence, bases: Optional[Sequence] = None):
        """BinaryConv.do (conv/j2t/impl.go:38-91) for a batch with the Go-side
        context: per message the HTTP request (EnableHttpMapping) and the
        request Base (EnableThriftBase). The host does what the reference's Go
        callbacks do (dynamicgo_amd.http):
          * writeRequestBaseToThrift: the Base field first;
          * handleHttpMappings for every struct with mapped fields, once per
            message (its bytes depend on the request and the struct only): the
            HTTP-mapping table the GPU writes from wherever the reference
            raises ERR_HM (dg_j2t_batch_host_hm, DG_F_HM_SPLIT);
          * an empty body: everything (impl.go:52-82);
          * the root's ERR_HM_END (F_TRACE_BACK): handleUnmatchedFields + STOP.
        Returns (outputs, errors): errors[i] is None, a J2TError (native
        status) or an http.ConvError."""
        self._check_opts()
        o = self.opts
        td = self._td(desc)
        n = len(msgs)
        bases = list(bases) if bases is not None else [None] * n
        if len(reqs) != n or len(bases) != n:
            raise ValueError("one request and one base (or None) per message")
        flags0 = to_flags(o)
        sd = td.struct if td.type == 12 else None
        flat = self._flat(td)
        hx = H.HMContext(o, self._nested(flags0))
        hm_structs = [x for x in flat.structs if x.hms] if o.EnableHttpMapping else []
        n_hm = len(hm_structs)
        outs: List[Optional[bytes]] = [None] * n
        errs: List[Optional[Exception]] = [None] * n
        prefix = [b""] * n
        rows = {}       # message -> its n_hm (off, len, mask) entries
        hm_err = {}     # (message, slot) -> the host's error for that struct
        hm_bytes = bytearray()
        groups = {}     # flag word -> message indices for the GPU
        rb = None
        if o.EnableThriftBase and sd is not None:
            rb = next((f for f in sorted(sd.fields, key=lambda f: f.id) if f.is_request_base), None)
        for i, src in enumerate(msgs):
            req = reqs[i]
            fl = flags0
            try:
                if o.EnableHttpMapping and req is None:
                    raise H.ConvError("ErrInvalidParam", "EnableHttpMapping but no http response in context")
                pre = b""
                if rb is not None:
                    b, no_write = H.write_request_base(bases[i], rb, src, o.MergeBaseFunc)
                    pre += b
                    if no_write:
                        fl |= F_NO_WRITE_BASE
                if len(src) == 0:
                    out = pre
                    if o.EnableHttpMapping and req is not None and sd is not None:
                        out += hx.empty_body(req, sd)
                    else:
                        out += b"\x00"
                    outs[i] = out
                    continue
            except H.ConvError as e:
                errs[i] = e
                continue
            if n_hm:
                row = []
                for j, hsd in enumerate(hm_structs):
                    try:
                        b, mask, _ = hx.handle_http_mappings(req, hsd, False)
                        row.append((len(hm_bytes), len(b), mask))
                        hm_bytes += b
                    except H.ConvError as e:
                        row.append((0, 0xFFFFFFFF, 0))  # DG_HM_ERR
                        hm_err[(i, j)] = e
                rows[i] = row
                fl |= F_HM_SPLIT
            prefix[i] = pre
            groups.setdefault(fl, []).append(i)
        order = sorted(sd.fields, key=lambda f: f.id) if sd is not None else []
        for fl, idx in groups.items():
            sub = [msgs[i] for i in idx]
            split = bool(fl & F_HM_SPLIT)
            sub_rows = [rows[i] for i in idx] if split else None
            out_k, rets = self._host_cb(flat, sub, fl, sub_rows, n_hm if split else 0, bytes(hm_bytes) if split else b"")
            sub_errs = [None] * len(idx)
            if fl & (F_VALUE_MAPPING | F_HM_SPLIT):
                def hm_end(k, hsd, ids, idx=idx):  # a nested struct's ERR_HM_END (top = true)
                    return hx.handle_unmatched_fields(reqs[idx[k]], hsd, ids, True) + b"\x00"
                self._serve_callbacks(flat, sub, fl, out_k, rets, sub_errs, sub_rows, n_hm if split else 0,
                                      bytes(hm_bytes) if split else b"", hm_end)
            for k, i in enumerate(idx):
                if sub_errs[k] is not None:
                    errs[i] = sub_errs[k]
                    continue
                r = int(rets[k])
                body = out_k[k]
                if r == 0:
                    outs[i] = prefix[i] + body
                elif (r & 0xFF) == DG_ST_HM_END:
                    # the root's ERR_HM_END: the unmatched fields are the set bits of
                    # the requires words behind the partial output (field index in id order)
                    w = r >> 40
                    part, words = body[:len(body) - 8 * w], body[len(body) - 8 * w:]
                    ids = []
                    for j in range(w):
                        bits = int.from_bytes(words[8 * j:8 * j + 8], "big")
                        ids += [order[64 * j + b].id for b in range(64)
                                if (bits >> b) & 1 and 64 * j + b < len(order)]
                    ids = [x for x in ids if not sd.field_by_id(x).is_request_base]
                    try:
                        outs[i] = prefix[i] + part + hx.handle_unmatched_fields(reqs[i], sd, ids, True) + b"\x00"
                    except H.ConvError as e:
                        errs[i] = e
                elif (r & 0xFF) == DG_ST_HM_ERR:
                    errs[i] = hm_err[(i, r >> 40)]
                else:
                    errs[i] = J2TError(r, explain_native_error(r, msgs[i]))
        return outs, errs

    def do_batch_hm_split(self, desc, msgs: Sequence[bytes], prefixes: Sequence[bytes]):
        """The root-only pre-split (DG_F_HM_SPLIT without a table): the caller
        has run handleHttpMappings (conv/j2t/impl.go:243-292) for the ROOT
        struct and passes prefixes[i], its mapped fields' Thrift bytes, every
        value found; the GPU converts the bodies (mapped keys skipped, mapped
        fields counted as set) and each result is prefix + body. A nested
        struct with mapped fields returns ERR_HM (19): do_batch_http serves
        those."""
        if len(prefixes) != len(msgs):
            raise ValueError("one prefix per message")
        outs, rets = self.do_batch(desc, msgs, extra_flags=F_HTTP_MAPPING | F_HM_SPLIT)
        # a null body converts to nothing: no struct, no mapped fields
        return [p + o if int(r) == 0 and o else b"" for p, o, r in zip(prefixes, outs, rets)], rets

    def do_batch(self, desc, msgs: Sequence[bytes], extra_flags: int = 0, chunks: int = 0,
                 out_cap: Optional[int] = None) -> Tuple[List[bytes], np.ndarray]:
        """Batch of independent messages -> (outputs, packed statuses).
        chunks > 0 streams the batch through dg_j2t_pipeline_host in that many
        overlapped pieces (uploads, kernels and downloads of neighbouring
        chunks in flight at once); out_cap overrides the first output
        capacity (the DG_E_NOMEM retry then takes out_need). Non-inline
        value mappings are served (ERR_VM_END); one whose callback failed
        keeps status ERR_VM_END (do_batch_errors returns its error)."""
        outs, rets, _ = self._do_batch(desc, msgs, extra_flags, chunks, out_cap)
        return outs, rets

    def _do_batch(self, desc, msgs: Sequence[bytes], extra_flags: int = 0, chunks: int = 0,
                  out_cap: Optional[int] = None):
        self._check_opts()
        flat = self._flat(desc)
        ctx = self._ctx()
        n = len(msgs)
        lens = np.fromiter((len(m) for m in msgs), dtype=np.uint64, count=n)
        in_off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(lens, out=in_off[1:])
        arena = np.frombuffer(b"".join(msgs) + b"\0" * 16, dtype=np.uint8)
        rets = np.zeros(max(n, 1), dtype=np.uint64)
        out_off = np.zeros(n + 1, dtype=np.uint64)
        cap = int(lens.sum()) * 4 + 64 * n + 64 if out_cap is None else out_cap
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        need = C.c_uint64(0)
        L = _lib.lib()
        flags = to_flags(self.opts) | extra_flags
        if flags & F_VALUE_MAPPING:
            flags |= F_CB_COLLECT  # every value-mapping callback of a pass at once

        def call(out, cap):
            if chunks > 0:
                return L.dg_j2t_pipeline_host(ctx.h, ctx.desc(flat), flat.root_type, arena.ctypes.data,
                                              in_off.ctypes.data, n, flags, chunks, out.ctypes.data, cap,
                                              out_off.ctypes.data, rets.ctypes.data, C.byref(need))
            return L.dg_j2t_batch_host(ctx.h, ctx.desc(flat), flat.root_type, arena.ctypes.data, in_off.ctypes.data,
                                       n, flags, out.ctypes.data, cap, out_off.ctypes.data,
                                       rets.ctypes.data, C.byref(need))
        rc = call(out, cap)
        if rc == -3 and need.value > cap:
            cap = int(need.value) + 64
            out = np.zeros(cap, dtype=np.uint8)
            rc = call(out, cap)
        _lib.check(rc)
        outs = [out[int(out_off[i]):int(out_off[i + 1])].tobytes() for i in range(n)]
        rets = rets[:n]
        vm_errs = {}
        if flags & F_VALUE_MAPPING and any((int(r) & 0xFF) in _CB_CODES for r in rets):
            errs = [None] * n
            self._serve_callbacks(flat, msgs, flags, outs, rets, errs)
            vm_errs = {i: e for i, e in enumerate(errs) if e is not None}
        for i in range(n):
            if int(rets[i]) != 0:
                outs[i] = b""
        return outs, rets, vm_errs

    def do_device(self, desc, json, in_off, out, out_off, out_len, ret, pending=None, stream=None):
        """Device-resident batch over torch CUDA tensors (uint8/int64/int32).

        json: uint8[>= in_off[-1] + 16]; in_off/out_off: int64[n+1];
        out: uint8 arena; out_len: int32[n]; ret: int64[n]. Asynchronous on
        `stream` (a torch.cuda.Stream), by default torch's current stream of
        the tensors' device, so the launch is ordered after whatever torch
        enqueued to fill the inputs and before whatever reads the outputs.
        """
        self._check_opts()
        flat = self._flat(desc)
        ctx = self._ctx()
        n = in_off.numel() - 1
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(json.device)
        s = stream.cuda_stream
        _lib.check(_lib.lib().dg_j2t_batch_device(
            ctx.h, ctx.desc(flat), flat.root_type, json.data_ptr(), in_off.data_ptr(), n,
            to_flags(self.opts), out.data_ptr(), out_off.data_ptr(), out_len.data_ptr(), ret.data_ptr(),
            pending.data_ptr() if pending is not None else None, s))


def new_binary_conv(opts: Optional[Options] = None) -> BinaryConv:
    """j2t.NewBinaryConv (conv/j2t/conv.go:36)."""
    return BinaryConv(opts)


class Aggregator:
    """BinaryConv.Do for many concurrent callers (dg_agg): each call blocks its
    thread; a flusher converts whatever is queued as one device batch as soon
    as max_batch messages wait or the oldest has waited max_wait_us. The
    shape a cgo shim gives the reference's goroutine-parallel Do
    (conv/j2t/conv_timing_test.go:76-99)."""

    def __init__(self, desc, opts: Optional[Options] = None, max_batch: int = 4096, max_wait_us: int = 200,
                 ctx: Optional[Context] = None, max_bytes: Optional[int] = None):
        self.conv = BinaryConv(opts, ctx=ctx)
        self.flat = self.conv._flat(desc)
        c = self.conv._ctx()
        h = C.c_void_p()
        if max_bytes is None:
            _lib.check(_lib.lib().dg_agg_create(c.h, c.desc(self.flat), self.flat.root_type,
                                                to_flags(self.conv.opts), max_batch, max_wait_us, C.byref(h)))
        else:
            _lib.check(_lib.lib().dg_agg_create2(c.h, c.desc(self.flat), self.flat.root_type,
                                                 to_flags(self.conv.opts), max_batch, max_bytes, max_wait_us,
                                                 C.byref(h)))
        self.h = h

    def do(self, jbytes: bytes) -> Optional[bytes]:
        """BinaryConv.Do through the aggregator (thread-safe; ctypes drops the
        GIL for the blocking call)."""
        L = _lib.lib()
        cap = 4 * len(jbytes) + 64
        for _ in range(2):
            out = C.create_string_buffer(max(cap, 1))
            ol, ret = C.c_size_t(0), C.c_uint64(0)
            rc = L.dg_agg_do(self.h, jbytes, len(jbytes), out, cap, C.byref(ol), C.byref(ret))
            if rc == -3 and ol.value > cap:  # DG_E_NOMEM: retry with the size it needs
                cap = ol.value
                continue
            _lib.check(rc)
            if ret.value != 0:
                raise J2TError(int(ret.value), explain_native_error(int(ret.value), jbytes))
            return out.raw[:ol.value] or None
        raise J2TError(0, "aggregator: output did not fit")

    def drive(self, msgs: Sequence[bytes], threads: int = 16, window: int = 256):
        """The reference's b.RunParallel over Do (conv/j2t/conv_timing_test.go:
        76-99) from C: `threads` OS threads, each with up to `window` calls in
        flight (dg_agg_drive). Returns (outputs, statuses, latency ns per
        message, wall seconds); statuses are the packed status words."""
        n = len(msgs)
        lens = np.fromiter((len(m) for m in msgs), dtype=np.uint64, count=n)
        in_off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(lens, out=in_off[1:])
        arena = np.frombuffer(b"".join(msgs) + b"\0" * 16, dtype=np.uint8)
        out_off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(lens * 4 + 4096, out=out_off[1:])
        out = np.zeros(int(out_off[-1]) + 64, dtype=np.uint8)
        out_len = np.zeros(max(n, 1), dtype=np.uint64)
        rets = np.zeros(max(n, 1), dtype=np.uint64)
        lat = np.zeros(max(n, 1), dtype=np.uint32)
        secs = C.c_double(0)
        _lib.check(_lib.lib().dg_agg_drive(self.h, arena.ctypes.data, in_off.ctypes.data, n, threads, window,
                                           out.ctypes.data, out_off.ctypes.data, out_len.ctypes.data,
                                           rets.ctypes.data, lat.ctypes.data, C.byref(secs)))
        outs = [out[int(out_off[i]):int(out_off[i]) + int(out_len[i])].tobytes() for i in range(n)]
        return outs, rets[:n], lat[:n], secs.value

    def set_knob(self, name: str, value: int):
        """dg_agg_set_knob: "depth" (seal as soon as fewer than depth batches
        convert; for callers that park instead of blocking), "max_wait_us"."""
        _lib.check(_lib.lib().dg_agg_set_knob(self.h, name.encode(), int(value)))

    def gateway(self, msgs: Sequence[bytes], callers: int = 1024, workers: int = 16):
        """The gateway shape (dg_agg_gateway_drive): `callers` logical callers
        with one call in flight each -- goroutines in Do -- multiplexed over
        `workers` OS threads, woken per converted generation by one poller
        (dg_agg_wait_gen). Returns (outputs, statuses, latency ns of every 8th
        message, wall seconds, stats [parks, retries, wake-ups, callers, worker ns in
        wait, in submit, idle, in all])."""
        n = len(msgs)
        lens = np.fromiter((len(m) for m in msgs), dtype=np.uint64, count=n)
        in_off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(lens, out=in_off[1:])
        arena = np.frombuffer(b"".join(msgs) + b"\0" * 16, dtype=np.uint8)
        out_off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(lens * 4 + 4096, out=out_off[1:])
        out = np.zeros(int(out_off[-1]) + 64, dtype=np.uint8)
        out_len = np.zeros(max(n, 1), dtype=np.uint64)
        rets = np.zeros(max(n, 1), dtype=np.uint64)
        lat = np.zeros(max(n, 1), dtype=np.uint32)
        st = np.zeros(8, dtype=np.uint64)
        secs = C.c_double(0)
        _lib.check(_lib.lib().dg_agg_gateway_drive(self.h, arena.ctypes.data, in_off.ctypes.data, n, workers, callers,
                                                   out.ctypes.data, out_off.ctypes.data, out_len.ctypes.data,
                                                   rets.ctypes.data, lat.ctypes.data, C.byref(secs), st.ctypes.data))
        outs = [out[int(out_off[i]):int(out_off[i]) + int(out_len[i])].tobytes() for i in range(n)]
        return outs, rets[:n], lat[:n], secs.value, [int(v) for v in st]

    def stats(self) -> Tuple[int, int]:
        """(batches flushed, messages converted)."""
        b, m = C.c_uint64(0), C.c_uint64(0)
        _lib.check(_lib.lib().dg_agg_stats(self.h, C.byref(b), C.byref(m)))
        return int(b.value), int(m.value)

    def profile(self) -> List[int]:
        """dg_agg_profile's 16 counters (include/dgj2t.h); [11]: calls
        converted alone (no part for their thread, or longer than a part)."""
        out = (C.c_uint64 * 16)()
        _lib.check(_lib.lib().dg_agg_profile(self.h, out, 16))
        return [int(v) for v in out]

    def close(self):
        if self.h:
            _lib.lib().dg_agg_destroy(self.h)
            self.h = None


# ---- HTTPConv (conv/j2t/http_conv.go) ----
ENCODING_THRIFT_BINARY = 0  # meta.EncodingThriftBinary
MSG_CALL = 1                # thrift.CALL (thrift/binary.go:55)
VERSION_1 = 0x80010000      # thrift/descriptor.go:30


def get_binary_message_header_and_footer(method: str, msg_type: int, struct_id: int,
                                         seq_id: int = 0) -> Tuple[bytes, bytes]:
    """thrift.GetBinaryMessageHeaderAndFooter (thrift/binary.go:137-175):
    WriteMessageBegin (i32 VERSION_1|type, string name, i32 seq) +
    WriteStructBegin (nothing) + WriteFieldBegin(STRUCT, id); the footer is
    WriteFieldEnd (nothing) + WriteStructEnd (STOP) + WriteMessageEnd (nothing)."""
    import struct as _s
    name = method.encode()
    hdr = (_s.pack(">I", (VERSION_1 | msg_type) & 0xFFFFFFFF) + _s.pack(">I", len(name)) + name +
           _s.pack(">i", seq_id) + bytes([12]) + _s.pack(">h", struct_id))
    return hdr, b"\x00"


class HTTPConv:
    """j2t.HTTPConv (conv/j2t/http_conv.go:28-114): the request body converted
    with EnableHttpMapping and wrapped in the Thrift message header/footer of
    the method's first request field. ``do_batch`` frames on the GPU
    (dg_pack_device_framed)."""

    def __init__(self, proto: int, fn_desc, ctx: Optional[Context] = None):
        if proto != ENCODING_THRIFT_BINARY:
            raise ValueError("now only support binary protocol")
        first = fn_desc.request().struct.fields[0]
        if first.type.type != 12:
            raise ValueError("first request field doesn't have struct kind")
        self.proto = proto
        self.st = first.type
        self.top, self.bottom = get_binary_message_header_and_footer(fn_desc.name, MSG_CALL, first.id, 0)
        self.ctx = ctx

    def _conv(self, opts: Optional[Options]) -> BinaryConv:
        o = Options(**vars(opts)) if opts is not None else Options()
        o.EnableHttpMapping = True  # conv/j2t/http_conv.go:73
        return BinaryConv(o, ctx=self.ctx)

    def do(self, req, opts: Optional[Options] = None) -> bytes:
        """HTTPConv.Do: header + body + footer, or J2TError / http.ConvError.
        The request's mapped values are written by the host half
        (BinaryConv.do_batch_http)."""
        body = self._conv(opts).do(self.st, req.get_body(), req=req) or b""
        return self.top + body + self.bottom

    def do_into(self, req, buf: bytearray, opts: Optional[Options] = None):
        """HTTPConv.DoInto: appends header + body + footer to buf."""
        out = self.do(req, opts)
        buf.extend(out)

    def do_batch(self, reqs: Sequence, opts: Optional[Options] = None):
        """Many requests. A root without HTTP-mapped fields is converted and
        framed on the GPU (dg_pack_device_framed); one with them goes through
        the host half (BinaryConv.do_batch_http) and is framed here. Returns
        (framed message per request (b"" where it failed), errors: None, a
        J2TError or an http.ConvError)."""
        cv = self._conv(opts)
        if self.st.struct.hms or cv.opts.EnableThriftBase or any(len(r.get_body()) == 0 for r in reqs):
            outs, errs = cv.do_batch_http(self.st, [r.get_body() for r in reqs], list(reqs))
            return [self.top + (o or b"") + self.bottom if e is None else b"" for o, e in zip(outs, errs)], errs
        outs, rets = self._framed_on_gpu(cv, reqs)
        return outs, [None if int(r) == 0 else J2TError(int(r), explain_native_error(int(r), q.get_body()))
                      for r, q in zip(rets, reqs)]

    def _framed_on_gpu(self, cv, reqs: Sequence):
        import torch
        ctx = cv._ctx()
        flat = cv._flat(self.st)
        bodies = [r.get_body() for r in reqs]
        n = len(bodies)
        lens = np.fromiter((len(b) for b in bodies), dtype=np.int64, count=n)
        in_off = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(lens, out=in_off[1:])
        slots = np.zeros(n + 1, dtype=np.int64)
        np.cumsum((lens * 4 + 64 + 7) & ~7, out=slots[1:])
        dev = torch.device("cuda", ctx.device)
        st = torch.cuda.current_stream(dev)
        d_json = torch.from_numpy(np.frombuffer(b"".join(bodies) + b"\0" * 64, dtype=np.uint8).copy()).to(dev)
        d_in = torch.from_numpy(in_off).to(dev)
        d_oo = torch.from_numpy(slots).to(dev)
        d_out = torch.empty(int(slots[-1]) + 64, dtype=torch.uint8, device=dev)
        d_ol = torch.zeros(n, dtype=torch.int32, device=dev)
        d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
        fx = len(self.top) + len(self.bottom)
        d_dst = torch.empty(int(slots[-1]) + fx * n + 64, dtype=torch.uint8, device=dev)
        d_doff = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        L = _lib.lib()
        _lib.check(L.dg_j2t_batch_device(ctx.h, ctx.desc(flat), flat.root_type, d_json.data_ptr(), d_in.data_ptr(), n,
                                         to_flags(cv.opts), d_out.data_ptr(), d_oo.data_ptr(), d_ol.data_ptr(),
                                         d_ret.data_ptr(), None, st.cuda_stream))
        _lib.check(L.dg_pack_device_framed(ctx.h, d_out.data_ptr(), d_oo.data_ptr(), d_ol.data_ptr(), d_ret.data_ptr(),
                                           n, self.top, len(self.top), self.bottom, len(self.bottom), d_dst.data_ptr(),
                                           d_doff.data_ptr(), st.cuda_stream))
        doff = d_doff.cpu().numpy()
        packed = d_dst[:int(doff[-1])].cpu().numpy().tobytes()
        rets = d_ret.cpu().numpy().astype(np.uint64)
        pending = [i for i in range(n) if (int(rets[i]) & 0xFF) == DG_ST_OUT_OVERFLOW]
        outs = [packed[int(doff[i]):int(doff[i + 1])] for i in range(n)]
        for i in pending:  # slot overflow: the exact-size host rerun
            try:
                outs[i] = self.do(reqs[i], cv.opts)
                rets[i] = 0
            except J2TError as e:
                outs[i], rets[i] = b"", e.ret
        return outs, rets


def HTTPRequest(body: bytes = b"", **kw) -> "H.HTTPRequest":
    """http.HTTPRequest (dynamicgo_amd.http) with the body first: url,
    headers, cookies, params, post_form as keyword arguments."""
    return H.HTTPRequest(body=body, **kw)
