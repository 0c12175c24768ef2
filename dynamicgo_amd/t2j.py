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
  * EnableHttpMapping (writeHttpValue, impl.go:515-588; handleUnsets
    :401-429): the device stops a message at each writeHttpValue call
    (DG_T2J_E_CALLBACK, the field and the value's position); here the call
    runs -- the value read by the mapping's encoding (Thrift bytes, text,
    the kitex string, or its JSON, which the device converts when asked) and
    HttpMapping.Response on the http.ResponseSetter -- and the message is
    converted again with the answer (taken / write to the JSON as well).
"""
from __future__ import annotations

import ctypes as C
import math
import struct as _st
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from . import http as H
from . import thrift as T
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
T2J_HM = 1 << 11

(E_READ, E_UNKNOWN_FIELD, E_DISMATCH_TYPE, E_UNSUPPORTED, E_NAN_INF, E_MISS_REQUIRED, E_NEEDS_HOST, E_DEPTH, E_WRITE,
 E_CONVERT, E_EXCEPTION, E_CALLBACK) = range(1, 13)

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
    base: a BaseResp is in the context (EnableThriftBase skips the field).
    EnableHttpMapping needs a ResponseSetter (Do, conv/t2j/conv.go:53-65)."""
    f = 0
    if o.EnableHttpMapping:
        f |= T2J_HM
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


# ------------------------------------------------------------ writeHttpValue
def f64toa(v: float) -> str:
    """json.EncodeFloat64 (internal/json/encoding.go:78, native f64toa
    native/fastfloat.c:349-404): integers below 2^53 in full, else the
    shortest round-trip digits as a decimal, or d.ddde[+-]x when the decimal
    exponent is < -6 or > 20; nothing for NaN and Inf."""
    if math.isnan(v) or math.isinf(v):
        return ""
    sign = "-" if math.copysign(1.0, v) < 0 else ""
    a = abs(v)
    if a == 0:
        return sign + "0"
    if a.is_integer() and a < 2.0 ** 53:
        return sign + str(int(a))
    mant, _, e = repr(a).partition("e")
    ip, _, fp = mant.partition(".")
    raw = (ip + fp).lstrip("0")
    digs = raw.rstrip("0")
    exp = (int(e) if e else 0) - len(fp) + (len(raw) - len(digs))
    nd = len(digs)
    dot = nd + exp
    if dot - 1 < -6 or dot - 1 > 20:
        x = dot - 1
        out = digs[0] + ("." + digs[1:] if nd > 1 else "") + "e" + ("-" if x < 0 else "+") + str(abs(x))
    elif dot <= 0:
        out = "0." + "0" * (-dot) + digs
    elif nd > dot:
        out = digs[:dot] + "." + digs[dot:]
    else:
        out = digs + "0" * (dot - nd)
    return sign + out


def _go_g(v: float) -> str:
    """strconv.FormatFloat(v, 'g', -1, 64), what fmt's %v prints."""
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "+Inf" if v > 0 else "-Inf"
    if v == 0:
        return "-0" if math.copysign(1.0, v) < 0 else "0"
    mant, _, e = repr(abs(v)).partition("e")
    ip, _, fp = mant.partition(".")
    raw = (ip + fp).lstrip("0")
    digs = raw.rstrip("0") or "0"
    exp = (int(e) if e else 0) - len(fp) + (len(raw) - len(digs))
    x = len(digs) + exp - 1  # decimal exponent of the first digit
    sign = "-" if v < 0 else ""
    # shortest 'g': %e when x < -4 or x >= eprec, eprec = 6 (strconv/ftoa.go)
    if x < -4 or x >= 6:
        m = digs[0] + ("." + digs[1:] if len(digs) > 1 else "")
        return sign + m + "e" + ("-" if x < 0 else "+") + ("%02d" % abs(x))
    dot = x + 1
    if dot <= 0:
        return sign + "0." + "0" * (-dot) + digs
    if len(digs) > dot:
        return sign + digs[:dot] + "." + digs[dot:]
    return sign + digs + "0" * (dot - len(digs))


def _go_f(v: float) -> str:
    """strconv.FormatFloat(v, 'f', -1, 64)."""
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "+Inf" if v > 0 else "-Inf"
    if v == 0:
        return "-0" if math.copysign(1.0, v) < 0 else "0"
    mant, _, e = repr(abs(v)).partition("e")
    ip, _, fp = mant.partition(".")
    raw = (ip + fp).lstrip("0")
    digs = raw.rstrip("0")
    exp = (int(e) if e else 0) - len(fp) + (len(raw) - len(digs))
    dot = len(digs) + exp
    sign = "-" if v < 0 else ""
    if dot <= 0:
        return sign + "0." + "0" * (-dot) + digs
    if len(digs) > dot:
        return sign + digs[:dot] + "." + digs[dot:]
    return sign + digs + "0" * (dot - len(digs))


class _Rd:
    """BinaryProtocol's reads over one buffer (thrift/binary.go:688-817)."""

    def __init__(self, b: bytes, p: int):
        self.b, self.p = b, p

    def next(self, k: int) -> bytes:
        if self.p + k > len(self.b):
            raise ThriftReadError("EOF")
        v = self.b[self.p:self.p + k]
        self.p += k
        return v

    def u8(self) -> int:
        return self.next(1)[0]

    def be(self, k: int, signed: bool = True) -> int:
        return int.from_bytes(self.next(k), "big", signed=signed)

    def string(self) -> bytes:
        n = self.be(4)
        if n < 0 or n > len(self.b) - self.p:
            raise ThriftReadError("invalid data length")
        return self.next(n)


def _encode_text(t: T.TypeDescriptor, rd: _Rd, o: Options) -> bytes:
    """ReadStringWithDesc = EncodeText(asJson false), the scalar cases
    (thrift/binary.go:834-905): the text of a non-complex value. A BYTE reads
    as Go's byte, so both ByteAsUint8 branches print it unsigned."""
    tt = t.type
    if tt == T.BOOL:
        return b"true" if rd.u8() == 1 else b"false"
    if tt == T.BYTE:
        return str(rd.u8()).encode()
    if tt in (T.I16, T.I32, T.I64):
        return str(rd.be({T.I16: 2, T.I32: 4, T.I64: 8}[tt])).encode()
    if tt == T.DOUBLE:
        return f64toa(_st.unpack(">d", rd.next(8))[0]).encode()
    if tt == T.STRING:
        v = rd.string()
        if not o.NoBase64Binary and t.is_binary():
            import base64
            return base64.b64encode(v)
        return bytes(v)
    raise H.ConvError("ErrUnsupportedType", "text encoding of type %d (no registered mapping reads it)" % tt)


def _read_any(t: T.TypeDescriptor, rd: _Rd, o: Options):
    """ReadAnyWithDesc (thrift/binary.go:1008-1166) into tagged Python values
    for the kitex string: ("i", int), ("f", float), ("b", bool), ("s",
    bytes), ("y", bytes) for binary, ("l", [...]), ("m", [(k, v)...])."""
    tt = t.type
    if tt == T.BOOL:
        return ("b", rd.u8() == 1)
    if tt == T.BYTE:
        v = rd.u8()
        return ("i", v if o.ByteAsUint8 else (v - 256 if v > 127 else v))
    if tt in (T.I16, T.I32, T.I64):
        return ("i", rd.be({T.I16: 2, T.I32: 4, T.I64: 8}[tt]))
    if tt == T.DOUBLE:
        return ("f", _st.unpack(">d", rd.next(8))[0])
    if tt == T.STRING:
        return ("y" if t.is_binary() else "s", bytes(rd.string()))
    if tt in (T.LIST, T.SET):
        et, n = rd.u8(), rd.be(4)
        if et != t.elem.type:
            raise H.ConvError("ErrConvert", "dismatched primitive types")
        return ("l", [_read_any(t.elem, rd, o) for _ in range(max(n, 0))])
    if tt == T.MAP:
        kt, vt, n = rd.u8(), rd.u8(), rd.be(4)
        if vt != t.elem.type or kt != t.key.type:
            raise H.ConvError("ErrConvert", "dismatched primitive types")
        if kt not in (T.STRING, T.BYTE, T.I16, T.I32, T.I64, T.BOOL, T.DOUBLE):
            raise H.ConvError("ErrUnsupportedType", "kitex string of a map keyed by pointers (unordered in Go)")
        m = {}
        for _ in range(max(n, 0)):
            if kt == T.STRING:
                k = ("s", bytes(rd.string()))
            elif kt in (T.BYTE, T.I16, T.I32, T.I64):  # ReadInt: signed
                k = ("i", rd.be({T.BYTE: 1, T.I16: 2, T.I32: 4, T.I64: 8}[kt]))
            else:
                k = _read_any(t.key, rd, o)
            m[k] = _read_any(t.elem, rd, o)  # a repeated key: the last value
        return ("m", list(m.items()))
    if tt == T.STRUCT:
        m = {}
        while True:
            ft = rd.u8()
            if ft == 0:
                return ("m", list(m.items()))
            fid = rd.be(2)
            f = t.struct.field_by_id(fid)
            if f is None:
                if o.DisallowUnknownField:
                    raise H.ConvError("ErrUnknownField", "unknown field %d" % fid)
                rd.p = _skip(rd.b, rd.p, ft)
                continue
            m[("s", f.alias.encode())] = _read_any(f.type, rd, o)
    raise H.ConvError("ErrUnsupportedType", "unsupported type %d" % tt)


def _go_v(x) -> bytes:
    """fmt's %v of what ReadAnyWithDesc returns (maps printed key-sorted)."""
    k, v = x
    if k == "i":
        return str(v).encode()
    if k == "f":
        return _go_g(v).encode()
    if k == "b":
        return b"true" if v else b"false"
    if k == "s":
        return v
    if k == "y":
        return b"[" + b" ".join(str(c).encode() for c in v) + b"]"
    if k == "l":
        return b"[" + b" ".join(_go_v(e) for e in v) + b"]"
    items = sorted(v, key=lambda kv: (kv[0][1] if kv[0][0] != "b" else int(kv[0][1])))
    return b"map[" + b" ".join(_go_v(a) + b":" + _go_v(b) for a, b in items) + b"]"


def _kitex_to_string(x) -> bytes:
    """primitive.KitexToString (internal/primitive/impl.go:191-215)."""
    k, v = x
    if k == "f":
        return _go_f(v).encode()
    if k == "l":
        return b",".join(_kitex_to_string(e) for e in v)
    return _go_v(x)


def _is_complex(t: T.TypeDescriptor) -> bool:
    return t.type in (T.STRUCT, T.MAP, T.LIST, T.SET)


def _needs_json(field: T.FieldDescriptor, o: Options) -> bool:
    """Whether writeHttpValue reads the value as JSON (doRecurse, impl.go:
    561-574) for one of the field's mappings."""
    return _is_complex(field.type) and not o.UseKitexHttpEncoding and \
        any(H.mapping_encoding(k) == H.ENCODING_JSON for k, _ in field.http_mappings)


def _empty_json(t: T.TypeDescriptor, b: bytes, o: Options) -> bytes:
    """doRecurse of a handleUnsets default (WriteDefaultOrEmpty bytes) of a
    container type: empty containers only; other constants are not
    restated here (parity unpinned)."""
    if t.type in (T.LIST, T.SET) and b[1:5] == b"\0\0\0\0":
        return b"[]"
    if t.type == T.MAP and b[2:6] == b"\0\0\0\0":
        return b"{}"
    if t.type == T.STRUCT and b == b"\0":
        for f in sorted(t.struct.fields, key=lambda f: f.id):
            if t.struct.requires.get(f.id, False) or f.default_value is not None or \
                    o.WriteDefaultField or o.WriteOptionalField:
                raise H.ConvError("ErrUnsupportedType", "JSON of an unset mapped struct with fields to write "
                                  "(not restated; parity unpinned)")
        return b"{}"
    raise H.ConvError("ErrUnsupportedType", "JSON of a container constant for an unset mapped field "
                      "(not restated; parity unpinned)")


def write_http_value(o: Options, resp, field: T.FieldDescriptor, buf: bytes, p: int,
                     json_val: Optional[bytes]) -> Tuple[bool, int]:
    """writeHttpValue (conv/t2j/impl.go:515-588) with the value at buf[p:]:
    (ok, the position after what it read). json_val: the value's JSON when
    _needs_json (the device's conversion, or _empty_json's). Raises the error
    the reference returns (read failures, a Response error unless
    OmitHttpMappingErrors)."""
    thrift_val = text_val = None
    rd = _Rd(buf, p)
    ok = False
    for kind, value in field.http_mappings:
        enc = H.mapping_encoding(kind)
        if enc == H.ENCODING_THRIFT_BINARY:
            if thrift_val is None:
                s0 = rd.p
                try:
                    rd.p = _skip(rd.b, rd.p, field.type.type, 1023)
                except ThriftReadError as e:
                    raise H.ConvError("ErrRead", "", e)
                thrift_val = bytes(rd.b[s0:rd.p])
            val = thrift_val
        elif enc == H.ENCODING_TEXT or not _is_complex(field.type):
            if text_val is None:
                try:
                    text_val = _encode_text(field.type, rd, o)
                except ThriftReadError as e:
                    raise H.ConvError("ErrRead", "reading thrift value of '%s' failed, thrift pos:%d" %
                                      (field.name, rd.p), e)
            val = text_val
        elif o.UseKitexHttpEncoding:
            if text_val is None:
                try:
                    text_val = _kitex_to_string(_read_any(field.type, rd, o))
                except ThriftReadError as e:
                    raise H.ConvError("ErrRead", "reading thrift value of '%s' failed, thrift pos:%d" %
                                      (field.name, rd.p), e)
            val = text_val
        else:  # EncodingJSON
            if json_val is None:
                raise H.ConvError("ErrUnsupportedType", "JSON value of '%s' read twice (not restated)" % field.name)
            val = json_val
        err = H.mapping_response(kind, value, resp, field, val)
        if err is None:
            ok = True
            break
        if not o.OmitHttpMappingErrors:
            raise err
    return ok, rd.p


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
        errors) with errors[i] None, T2JError, T2JException, ThriftReadError
        or http.ConvError (the HTTP mapping's Go-side errors). resps: each
        message's http.ResponseSetter (EnableHttpMapping needs one, Do
        conv/t2j/conv.go:53-65); bases: its BaseResp (EnableThriftBase)."""
        n = len(msgs)
        resps = list(resps) if resps is not None else [None] * n
        bases = list(bases) if bases is not None else [None] * n
        hm = bool(self.opts.EnableHttpMapping)
        errs: List[Optional[Exception]] = [None] * n
        outs: List[bytes] = [b""] * n
        rets = np.zeros(max(n, 1), dtype=np.uint64)
        aux: List[Optional[int]] = [None] * n
        pending = []
        for i in range(n):
            if hm and resps[i] is None:
                errs[i] = H.ConvError("ErrInvalidParam", "no http response in context")
            else:
                pending.append(i)
        answers = {i: bytearray() for i in pending} if hm else None
        flat = self._flat(desc) if hm else None
        while pending:
            nxt = []
            # readResponseBase skips the field only when the context holds a
            # BaseResp (conv/t2j/impl.go:54-58, 120-127): messages with and
            # without one run as separate launches with their own options
            for with_base in (True, False):
                grp = [i for i in pending if (bases[i] is not None) == with_base]
                if not grp:
                    continue
                o, r, a = self._batch(desc, [msgs[i] for i in grp], with_base,
                                      [answers[i] for i in grp] if hm else None)
                for k, i in enumerate(grp):
                    rr = int(r[k])
                    if hm and (rr & 0xFF) == E_CALLBACK:
                        try:
                            self._serve(flat, msgs[i], resps[i], answers[i], o[k])
                            nxt.append(i)
                        except (H.ConvError, ValueError, ThriftReadError) as e:
                            errs[i] = e
                        continue
                    outs[i], rets[i] = o[k], rr
                    aux[i] = int(a[k]) if a is not None else None
            pending = sorted(nxt)
        for i in range(n):
            if errs[i] is not None:
                outs[i] = b""
                continue
            r = int(rets[i])
            if (r & 0xFF) == E_EXCEPTION:
                errs[i], outs[i] = T2JException(outs[i]), b""
                continue
            if r != 0:
                errs[i] = T2JError(r)
                continue
            if bases[i] is not None and aux[i] is not None and aux[i] != 2**64 - 1:
                lo, hi = aux[i] & 0xFFFFFFFF, aux[i] >> 32
                try:
                    bases[i].fast_read(bytes(msgs[i][lo:hi]))  # readResponseBase's FastRead
                except ThriftReadError as e:
                    errs[i], outs[i] = e, b""
        return outs, errs

    def _serve(self, flat: FlatDescriptor, msg: bytes, resp, answers: bytearray, rec: bytes):
        """One writeHttpValue call the device stopped at (DG_T2J_E_CALLBACK,
        include/dgj2t_defs.h): run it and record the answer for the rerun."""
        w0, w1 = _st.unpack_from("<QQ", rec, len(rec) - 16)
        payload = bytes(rec[:-16])
        kind, has_resp, idx, fi = w0 & 0xFF, (w0 >> 8) & 1, (w0 >> 16) & 0xFFFF, w0 >> 32
        s0 = w1 & 0xFFFFFFFF
        field = flat.fields[fi]
        o = self.opts
        if kind == 1:  # a mapped field's value (impl.go:132-142, 296-306)
            done = idx < len(answers) and answers[idx] == 2
            if not done:
                if idx != len(answers):
                    raise H.ConvError("ErrConvert", "callback %d out of order (%d answers)" % (idx, len(answers)))
                if _needs_json(field, o):
                    answers.append(2)  # the device converts the value first
                    return
            try:
                ok, _ = write_http_value(o, resp, field, msg, s0, payload if done else None)
            except H.ConvError as e:
                raise H.ConvError(e.behavior, "mapping field %s failed: %s" % (field.name, e))
            except ValueError as e:  # a Response's plain error: unwrapError -> ErrConvert
                raise H.ConvError("ErrConvert", "mapping field %s failed" % field.name, e)
            del answers[idx:]
            answers.append(1 if (o.WriteHttpValueFallback and not ok) else 0)
            return
        # kind 2: handleUnsets (impl.go:401-429), the default or empty value
        if idx != len(answers):
            raise H.ConvError("ErrConvert", "callback %d out of order (%d answers)" % (idx, len(answers)))
        dflt = H.write_default_or_empty(field)
        jv = _empty_json(field.type, dflt, o) if _needs_json(field, o) else None
        ok, _ = write_http_value(o, resp if has_resp else None, field, dflt, 0, jv)
        answers.append(0 if ok else 1)

    def do_batch(self, desc, msgs: Sequence[bytes]) -> Tuple[List[bytes], np.ndarray]:
        """Batch of independent Thrift messages -> (JSON outputs, statuses).
        EnableHttpMapping needs the ResponseSetters: do_batch_errors."""
        if self.opts.EnableHttpMapping:
            raise ValueError("EnableHttpMapping: use do_batch_errors with the ResponseSetters")
        outs, rets, _ = self._batch(desc, msgs)
        return outs, rets

    def _batch(self, desc, msgs: Sequence[bytes], with_base: bool = False, answers=None):
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
        cb = None
        if answers is not None:
            tab = (_lib.VMEntry * max(n, 1))()
            blob = bytearray()
            for k, a in enumerate(answers):
                tab[k].off, tab[k].count = len(blob), len(a)
                blob += a
            ab = np.frombuffer(bytes(blob) + b"\0" * 8, dtype=np.uint8)
            cb = _lib.CBTables(None, 0, C.cast(tab, C.c_void_p), ab.ctypes.data, len(blob))
        for _ in range(2):
            rc = L.dg_t2j_batch_host_cb(ctx.h, d, flat.root_type, arena.ctypes.data, in_off.ctypes.data, n, opts,
                                        out.ctypes.data, cap, out_off.ctypes.data, rets.ctypes.data,
                                        C.byref(need), aux.ctypes.data if aux is not None else None,
                                        C.byref(cb) if cb is not None else None)
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
        if self.opts.EnableHttpMapping:
            raise ValueError("EnableHttpMapping: use do_batch_errors with the ResponseSetters")
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


# ---------------------------------------------------------------- HTTPConv
REPLY, EXCEPTION = 2, 3  # thrift.TMessageType (thrift/binary.go:52-57)


def unwrap_binary_message(buf: bytes):
    """thrift.UnwrapBinaryMessage (thrift/binary.go:193-220): (name, type,
    seqID, the result field's id, its value bytes). Raises ThriftReadError
    ("invalid version" for a malformed header, as ReadMessageBegin
    reports every failure)."""
    rd = _Rd(bytes(buf), 0)
    try:
        size = rd.be(4)  # int32
        if size > 0 or (size & 0xFFFF0000) != 0x80010000:  # VERSION_MASK / VERSION_1
            raise ThriftReadError("invalid version")
        typ = size & 0xFF
        name = bytes(rd.string()).decode("utf-8", "surrogateescape")
        seq = rd.be(4)
    except ThriftReadError:
        raise ThriftReadError("invalid version")
    t = rd.u8()
    if t not in (0, 1, 2, 3, 4, 6, 8, 10, 11, 12, 13, 14, 15, 16, 17):
        raise ThriftReadError("invalid data type")
    fid = rd.be(2) if t != 0 else 0
    if t == 0:
        return name, typ, seq, fid, b""
    if rd.p > len(rd.b) - 1:
        raise ThriftReadError("EOF")
    return name, typ, seq, fid, bytes(rd.b[rd.p:len(rd.b) - 1])


class HTTPConv:
    """t2j.HTTPConv (conv/t2j/http_conv.go:29-122): a Thrift REPLY (or
    exception) message -> the http.ResponseSetter: mapped fields to headers,
    cookies and the status code, the JSON body to SetRawBody. The body is
    converted on the GPU with EnableHttpMapping (BinaryConv above)."""

    def __init__(self, proto: int, fn_desc, conv: Optional[BinaryConv] = None):
        if proto != H.ENCODING_THRIFT_BINARY:
            raise ValueError("protocol %r is not supported" % proto)
        res = fn_desc.response()
        if res is None or res.struct.field_by_id(0) is None:
            raise ValueError("response field is not found in function")
        self.st = res.struct
        self.conv = conv or BinaryConv()

    def _desc(self, tbytes: bytes):
        _, typ, _, fid, body = unwrap_binary_message(tbytes)
        if typ != REPLY:
            f = self.st.field_by_id(fid)
            if f is None:
                raise H.ConvError("ErrUnknownField", "exception field is not foud in function")
            return f.type, body
        if fid != 0:
            raise H.ConvError("ErrInvalidParam", "unexpected response field id %d" % fid)
        return self.st.field_by_id(0).type, body

    def do_batch(self, resps: Sequence, msgs: Sequence[bytes], opts: Optional[Options] = None):
        """Do over a batch: errors[i] None or the error; each response gets
        its body. Messages are grouped by result type, one GPU batch each."""
        import dataclasses
        o = dataclasses.replace(opts or Options(), EnableHttpMapping=True)
        self.conv.set_options(o)
        n = len(msgs)
        errs: List[Optional[Exception]] = [None] * n
        groups: Dict[int, Tuple[object, List[int], List[bytes]]] = {}
        for i, m in enumerate(msgs):
            try:
                td, body = self._desc(m)
            except ThriftReadError as e:
                errs[i] = H.ConvError("ErrRead", "", e)
                continue
            except H.ConvError as e:
                errs[i] = e
                continue
            g = groups.setdefault(id(td), (td, [], []))
            g[1].append(i)
            g[2].append(body)
        for td, idx, bodies in groups.values():
            outs, es = self.conv.do_batch_errors(td, bodies, [resps[i] for i in idx])
            for k, i in enumerate(idx):
                if es[k] is not None:
                    errs[i] = es[k]
                else:
                    resps[i].set_raw_body(outs[k] or b"")
        return errs

    def do(self, resp, tbytes: bytes, opts: Optional[Options] = None):
        """HTTPConv.Do (conv/t2j/http_conv.go:53-85)."""
        e = self.do_batch([resp], [tbytes], opts)[0]
        if e is not None:
            raise e

    def do_into(self, resp, tbytes: bytes, buf: bytearray, opts: Optional[Options] = None):
        """HTTPConv.DoInto (conv/t2j/http_conv.go:88-122): the body appended
        to buf as well."""
        self.do(resp, tbytes, opts)
        buf.extend(resp.body or b"")
