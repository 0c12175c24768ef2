"""The host half of conv/j2t's HTTP mapping.

The GPU converts JSON bodies; what the reference does in Go callbacks around
its native FSM stays on the host here, restated:

  http.RequestGetter / HTTPRequest    http/http.go:63-84, 86-300
  HTTP-mapping annotations            thrift/annotation/http_mapping.go:111-300
  tryGetValueFromHttp                 conv/j2t/impl.go:195-218
  writeStringValue                    conv/j2t/impl.go:107-151
  BinaryProtocol.DecodeText (text)    thrift/binary.go:1176-1296
  BinaryProtocol.WriteDefaultOrEmpty  thrift/binary.go:474-515
  handleHttpMappings                  conv/j2t/impl.go:243-292
  handleUnmatchedFields               conv/j2t/impl_amd64.go:71-115
  writeRequestBaseToThrift            conv/j2t/impl.go:155-193 (base.Base, thrift/base)

How the two halves meet (conv.BinaryConv.do_batch_http): for the ROOT
struct's mapped fields the host runs handleHttpMappings before the GPU
(the reference calls it at ERR_HM, right after the root's '{', so its bytes
come first); the GPU converts the body with DG_F_HM_SPLIT and a per-message
mask of the mapped fields the host wrote (their JSON keys are skipped,
native/thrift.c:725). With ReadHttpValueFallback a mapped field the request
lacks is read from the body instead, and a root field still unset at the
root's '}' comes back as DG_ST_HM_END with the root's remaining requires
bitmap: the host serves it like handleUnmatchedFields and writes the STOP.
"""
from __future__ import annotations

import base64 as _b64
import json as _json
import math
import re
import struct as _st
from typing import Dict, Iterable, List, Optional, Tuple
from urllib.parse import parse_qs, urlsplit

from . import thrift as T

# meta.Encoding (meta/encoding.go)
ENCODING_THRIFT_BINARY = 0
ENCODING_JSON = 1
ENCODING_TEXT = 2


class ConvError(Exception):
    """A Go-side conversion error (meta.Error): `behavior` names its
    meta.ErrorCode (ErrMissRequiredField, ErrConvert, ErrNotFound, ...)."""

    def __init__(self, behavior: str, msg: str, cause: Optional[Exception] = None):
        super().__init__(msg if cause is None else "%s: %s" % (msg, cause))
        self.behavior = behavior


# ---------------------------------------------------------------- requests
_TOKEN = frozenset(b"!#$%&'*+-.^_`|~0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ")


def _canon_header(k: str) -> str:
    """textproto.CanonicalMIMEHeaderKey: unchanged when a byte is not a token
    byte (validHeaderFieldByte), else upper case at the start and after each
    '-', lower case elsewhere."""
    b = k.encode("utf-8", "surrogateescape")
    if any(c not in _TOKEN for c in b):
        return k
    return "-".join(p[:1].upper() + p[1:].lower() for p in k.split("-"))


def _top_level_members(body: bytes) -> Optional[Dict[str, Tuple[int, int]]]:
    """Spans of the top-level members of a JSON object body (raw value text),
    like the lazy ast.Node of GetMapBody (http/http.go:246-270)."""
    s = body.decode("utf-8", "surrogateescape")
    dec = _json.JSONDecoder()
    i, n = 0, len(s)
    ws = " \t\r\n"
    while i < n and s[i] in ws:
        i += 1
    if i >= n or s[i] != "{":
        return None
    i += 1
    out: Dict[str, Tuple[int, int]] = {}
    while True:
        while i < n and s[i] in ws:
            i += 1
        if i < n and s[i] == "}":
            return out
        try:
            key, i = dec.raw_decode(s, i)
        except ValueError:
            return None
        while i < n and s[i] in ws:
            i += 1
        if i >= n or s[i] != ":":
            return None
        i += 1
        while i < n and s[i] in ws:
            i += 1
        try:
            _, j = dec.raw_decode(s, i)
        except ValueError:
            return None
        if key not in out:
            out[key] = (i, j)
        i = j
        while i < n and s[i] in ws:
            i += 1
        if i < n and s[i] == ",":
            i += 1
            continue
        if i < n and s[i] == "}":
            return out
        return None


class HTTPRequest:
    """http.HTTPRequest (http/http.go:86-300), the RequestGetter the
    HTTP-mapping annotations read: url query, path params, headers, cookies,
    post form, the raw body and its top-level members (GetMapBody)."""

    def __init__(self, method: str = "POST", url: str = "http://localhost/", body: bytes = b"",
                 headers: Optional[Iterable] = None, cookies: Optional[Dict[str, str]] = None,
                 params: Optional[Dict[str, str]] = None, post_form: Optional[Dict[str, str]] = None):
        self.method = method
        self.url = url
        self.body = bytes(body)
        self.headers: Dict[str, List[str]] = {}
        for k, v in (headers.items() if isinstance(headers, dict) else (headers or ())):
            self.add_header(k, v)
        self.cookies: Dict[str, str] = dict(cookies or {})
        self.params: Dict[str, str] = dict(params or {})
        self._post_form = dict(post_form) if post_form is not None else None
        self._map = None

    # http.Header.Add / Set
    def add_header(self, k: str, v: str):
        self.headers.setdefault(_canon_header(k), []).append(str(v))

    def set_header(self, k: str, v: str):
        self.headers[_canon_header(k)] = [str(v)]

    def add_cookie(self, name: str, value: str):
        self.cookies[name] = value

    # ---- RequestGetter ----
    def get_method(self) -> str:
        return self.method

    def get_host(self) -> str:
        return urlsplit(self.url).netloc

    def get_uri(self) -> str:
        return self.url

    def get_header(self, key: str) -> str:
        v = self.headers.get(_canon_header(key))
        return v[0] if v else ""

    def get_cookie(self, key: str) -> str:
        if key in self.cookies:
            return self.cookies[key]
        for line in self.headers.get("Cookie", ()):
            for part in line.split(";"):
                k, _, v = part.strip().partition("=")
                if k == key:
                    return v
        return ""

    def get_query(self, key: str) -> str:
        v = parse_qs(urlsplit(self.url).query, keep_blank_values=True).get(key)
        return v[0] if v else ""

    def get_param(self, key: str) -> str:
        return self.params.get(key, "")

    def _content_type(self) -> str:
        return self.get_header("Content-Type")

    def get_post_form(self, key: str) -> str:
        if self._post_form is not None:
            return self._post_form.get(key, "")
        if self._content_type() == "application/x-www-form-urlencoded":
            v = parse_qs(self.body.decode("utf-8", "replace"), keep_blank_values=True).get(key)
            return v[0] if v else ""
        return ""

    def get_map_body(self, key: str) -> str:
        ct = self._content_type()
        if ct == "application/json":
            if self._map is None:
                self._map = _top_level_members(self.body) or {}
            span = self._map.get(key)
            if span is None:
                return ""
            raw = self.body.decode("utf-8", "surrogateescape")[span[0]:span[1]]
            if raw[:1] == '"':
                try:
                    return _json.loads(raw)
                except ValueError:
                    return ""
            return raw
        if ct == "application/x-www-form-urlencoded":
            return self.get_post_form(key)
        return ""

    def get_body(self) -> bytes:
        return self.body


# ---------------------------------------------------------------- responses
def _sanitize_cookie_value(v: bytes) -> bytes:
    """net/http sanitizeCookieValue: bytes outside 0x20-0x7e, '"', ';' and
    '\\' dropped; quoted when it holds ' ' or ','."""
    v = bytes(c for c in v if 0x20 <= c < 0x7F and c not in b'";\\')
    if v and (b" " in v or b"," in v):
        return b'"' + v + b'"'
    return v


def cookie_string(name: str, value: bytes) -> str:
    """(&http.Cookie{Name, Value}).String() (net/http/cookie.go): "" for an
    invalid name (empty or a non-token rune), else name=sanitized value."""
    nb = name.encode("utf-8", "surrogateescape")
    if not nb or any(c not in _TOKEN for c in nb):
        return ""
    return name + "=" + _sanitize_cookie_value(value).decode("latin-1")


class HTTPResponse:
    """http.HTTPResponse (http/http.go:304-346), the ResponseSetter t2j's
    HTTP mapping writes: status code, headers (Set-Cookie lines for cookies),
    raw body. Values are Go strings: bytes, kept as str by surrogateescape."""

    def __init__(self):
        self.status_code = 0
        self.headers: Dict[str, List[str]] = {}
        self.body: Optional[bytes] = None

    def set_status_code(self, code: int):
        self.status_code = code

    def set_header(self, key: str, val: str):
        self.headers[_canon_header(key)] = [val]  # Header.Set

    def set_cookie(self, key: str, val: str):
        self.headers.setdefault("Set-Cookie", []).append(
            cookie_string(key, val.encode("utf-8", "surrogateescape")))

    def set_raw_body(self, body: bytes):
        self.body = bytes(body)

    def get_header(self, key: str) -> str:
        """Header.Get"""
        v = self.headers.get(_canon_header(key))
        return v[0] if v else ""

    def cookies(self) -> List[Tuple[str, str]]:
        """Response.Cookies() for the lines set_cookie writes: (name, value)
        with the quotes of a quoted value removed (readSetCookies)."""
        out = []
        for line in self.headers.get("Set-Cookie", ()):
            k, eq, v = line.partition("=")
            if not eq or not k:
                continue
            if len(v) > 1 and v[0] == '"' and v[-1] == '"':
                v = v[1:-1]
            out.append((k, v))
        return out


def _parse_atoi(s: str) -> int:
    """strconv.Atoi (base 10, int64 range)."""
    if not re.fullmatch(r"[+-]?[0-9]+", s):
        raise ValueError('strconv.Atoi: parsing %r: invalid syntax' % s)
    v = int(s)
    if not -(1 << 63) <= v < (1 << 63):
        raise ValueError('strconv.Atoi: parsing %r: value out of range' % s)
    return v


def mapping_response(kind: str, value: str, resp, field: T.FieldDescriptor, val: bytes) -> Optional[Exception]:
    """HttpMapping.Response (thrift/annotation/http_mapping.go:119-351): None
    when the value was set, else the error the Go method returns. resp None
    is a nil ResponseSetter (handleUnsets below the root): the Go methods that
    touch it panic there, raised here as an error whatever the options."""
    sval = bytes(val).decode("utf-8", "surrogateescape")
    if kind in ("api.header", "api.cookie", "api.raw_body", "api.http_code") and resp is None:
        raise ConvError("ErrConvert", "nil ResponseSetter (%s): the reference panics here" % kind)
    if kind == "api.header":
        resp.set_header(value, sval)
    elif kind == "api.cookie":
        resp.set_cookie(value, sval)
    elif kind == "api.raw_body":
        resp.set_raw_body(bytes(val))
    elif kind == "api.http_code":
        try:
            resp.set_status_code(_parse_atoi(sval))
        except ValueError as e:
            return e
    elif kind == "api.raw_uri":
        return None
    else:  # query, path, body, form, no_body_struct: errNotImplemented (register.go:74-76)
        name = {"api.query": "apiQuery", "api.path": "apiPath", "api.body": "apiBody", "api.form": "apiPostForm",
                "api.no_body_struct": "apiNoBodyStruct"}.get(kind, kind)
        return ConvError("ErrUnsupportedType", "%s not support http response!" % name)
    return None


# ---------------------------------------------------------------- annotations
def mapping_request(kind: str, value: str, req: HTTPRequest, field: T.FieldDescriptor) -> Optional[str]:
    """HttpMapping.Request (thrift/annotation/http_mapping.go:111-300): the
    value, or None where the Go method returns an error (not found /
    unsupported)."""
    if kind == "api.query":
        v = req.get_query(value)
    elif kind == "api.path":
        v = req.get_param(value)
    elif kind == "api.header":
        v = req.get_header(value)
    elif kind == "api.cookie":
        v = req.get_cookie(value)
    elif kind == "api.body":
        v = req.get_map_body(value)
    elif kind == "api.form":
        v = req.get_post_form(value)
    elif kind == "api.raw_body":
        return req.get_body().decode("utf-8", "surrogateescape")
    elif kind == "api.raw_uri":
        return req.get_uri()
    elif kind == "api.no_body_struct":
        return no_body_struct(req, field)
    else:  # api.http_code: response only
        return None
    return v if v != "" else None


def mapping_encoding(kind: str) -> int:
    """HttpMapping.Encoding(): Thrift binary for api.no_body_struct
    (http_mapping.go:350-352), JSON for the request-side others."""
    return ENCODING_THRIFT_BINARY if kind == "api.no_body_struct" else ENCODING_JSON


def no_body_struct(req: HTTPRequest, field: T.FieldDescriptor) -> Optional[str]:
    """apiNoBodyStruct.Request (thrift/annotation/http_mapping.go:299-344): the
    STRUCT field's value built from the request alone -- each of its mapped
    fields (HttpMappingFields order) with its first value found, or its
    default / empty value, then STOP -- as Thrift binary (returned as a str
    whose surrogateescape encoding is the bytes). The conv options come from
    the context in Go; none here: the zero Options (base64 on, unknown fields
    allowed). A value WriteStringWithDesc rejects leaves only its header
    (the Go code drops that error)."""
    if field.type.type != T.STRUCT:
        return None  # "apiNoBodyStruct only support STRUCT type"
    out = b""
    for f in field.type.struct.hms:
        val = None
        for kind, value in f.http_mappings:
            v = mapping_request(kind, value, req, f)
            if v is not None:
                val = v
                break
        out += field_begin(f)
        if val is None or val == "":
            out += write_default_or_empty(f)
        else:
            try:
                out += decode_text(val, f.type, False, True)
            except (ValueError, ConvError):
                pass
    out += b"\x00"
    return out.decode("utf-8", "surrogateescape")


def try_get_value_from_http(req: Optional[HTTPRequest], key: str) -> Tuple[str, bool, int]:
    """tryGetValueFromHttp conv/j2t/impl.go:195-218: url param -> query ->
    header -> cookie -> body member."""
    if req is None:
        return "", False, ENCODING_TEXT
    for get in (req.get_param, req.get_query, req.get_header, req.get_cookie, req.get_map_body):
        v = get(key)
        if v != "":
            return v, True, ENCODING_JSON
    return "", False, ENCODING_TEXT


# ---------------------------------------------------------------- Thrift writes
def field_begin(f: T.FieldDescriptor) -> bytes:
    return bytes([f.type.type]) + _st.pack(">h", f.id)


def write_empty(t: T.TypeDescriptor) -> bytes:
    """BinaryProtocol.WriteEmpty thrift/binary.go:483-515."""
    if t.type in (T.BOOL, T.BYTE):
        return b"\x00"
    if t.type == T.I16:
        return b"\x00" * 2
    if t.type in (T.I32, T.STRING):
        return b"\x00" * 4
    if t.type in (T.I64, T.DOUBLE):
        return b"\x00" * 8
    if t.type in (T.LIST, T.SET):
        return bytes([t.elem.type]) + b"\x00" * 4
    if t.type == T.MAP:
        return bytes([t.key.type, t.elem.type]) + b"\x00" * 4
    if t.type == T.STRUCT:
        return b"\x00"
    raise ConvError("ErrWrite", "invalid type")


def write_default_or_empty(f: T.FieldDescriptor) -> bytes:
    """BinaryProtocol.WriteDefaultOrEmpty thrift/binary.go:474-480."""
    if f.default_value is not None:
        return bytes(f.default_value)
    return write_empty(f.type)


_INT_RE = re.compile(r"[+-]?[0-9]+\Z")
_DEC_RE = re.compile(r"[+-]?([0-9]+\.?[0-9]*|\.[0-9]+)([eE][+-]?[0-9]+)?\Z")
_HEX_RE = re.compile(r"[+-]?0[xX]([0-9a-fA-F]+\.?[0-9a-fA-F]*|\.[0-9a-fA-F]+)[pP][+-]?[0-9]+\Z")


def parse_int(s: str) -> int:
    """strconv.ParseInt(s, 10, 64)."""
    if not _INT_RE.match(s):
        raise ValueError('strconv.ParseInt: parsing %r: invalid syntax' % s)
    v = int(s)
    if not -2**63 <= v < 2**63:
        raise ValueError('strconv.ParseInt: parsing %r: value out of range' % s)
    return v


def parse_float(s: str) -> float:
    """strconv.ParseFloat(s, 64): decimal and hex forms, inf/infinity/nan;
    overflow is an error (no underscores without a base prefix)."""
    low = s.lower()
    sign = -1.0 if low[:1] == "-" else 1.0
    body = low[1:] if low[:1] in "+-" else low
    if body in ("inf", "infinity"):
        return sign * math.inf
    if body == "nan" and low == body:
        return math.nan
    if _DEC_RE.match(s):
        v = float(s)
    elif _HEX_RE.match(s):
        m = s[1:] if s[:1] in "+-" else s
        v = float.fromhex(m) * (-1.0 if s[:1] == "-" else 1.0)
    else:
        raise ValueError('strconv.ParseFloat: parsing %r: invalid syntax' % s)
    if math.isinf(v):
        raise ValueError('strconv.ParseFloat: parsing %r: value out of range' % s)
    return v


def parse_bool(s: str) -> bool:
    """strconv.ParseBool."""
    if s in ("1", "t", "T", "TRUE", "true", "True"):
        return True
    if s in ("0", "f", "F", "FALSE", "false", "False"):
        return False
    raise ValueError('strconv.ParseBool: parsing %r: invalid syntax' % s)


def b64_std_decode(s: str) -> bytes:
    """base64.StdEncoding.DecodeString: padded standard alphabet, CR/LF skipped."""
    t = s.replace("\r", "").replace("\n", "")
    try:
        return _b64.b64decode(t.encode("latin-1"), validate=True)
    except Exception as e:  # binascii.Error / UnicodeEncodeError
        raise ValueError("illegal base64 data") from e


def decode_text(val: str, t: T.TypeDescriptor, disallow_unknown: bool, base64_binary: bool) -> bytes:
    """BinaryProtocol.DecodeText(val, desc, .., useFieldName=true, asJson=false)
    thrift/binary.go:1176-1296: the text form of an HTTP value as Thrift."""
    if t.type == T.STRING:
        raw = val.encode("utf-8", "surrogateescape")
        if base64_binary and t.is_binary():
            raw = b64_std_decode(val)
        return _st.pack(">I", len(raw)) + raw
    if t.type == T.BOOL:
        return b"\x01" if parse_bool(val) else b"\x00"
    if t.type in (T.BYTE, T.I16, T.I32, T.I64):
        v = parse_int(val)
        fmt, bits = {T.BYTE: (">B", 8), T.I16: (">H", 16), T.I32: (">I", 32), T.I64: (">Q", 64)}[t.type]
        return _st.pack(fmt, v & ((1 << bits) - 1))
    if t.type == T.DOUBLE:
        return _st.pack(">d", parse_float(val))
    if t.type in (T.LIST, T.SET):
        vs = val.split(",")
        out = bytes([t.elem.type]) + _st.pack(">I", len(vs))
        for v in vs:
            out += decode_text(v, t.elem, disallow_unknown, base64_binary)
        return out
    if t.type in (T.MAP, T.STRUCT):
        raise ValueError("not implemented")  # errNotImplemented: non-JSON text of a map/struct
    raise ValueError("dismatched primitive type")


def is_json_string(val: str) -> bool:
    """isJsonString conv/j2t/impl.go:93-105."""
    if len(val) < 2:
        return False
    c = 0
    while c < len(val) and val[c] in " \t\r\n":
        c += 1
    if c >= len(val):
        return False
    s, e = val[c], val[-1]
    return (s == "{" and e == "}") or (s == "[" and e == "]") or (s == '"' and e == '"')


def _is_complex(t: T.TypeDescriptor) -> bool:
    return t.type in (T.STRUCT, T.MAP, T.LIST, T.SET)


class HMContext:
    """What writeStringValue needs besides the field and value: the options
    and the nested converter for JSON-encoded complex values (the reference
    recurses into doImpl, conv/j2t/impl.go:140-145; here: a GPU batch)."""

    def __init__(self, opts, nested=None):
        self.opts = opts
        self.nested = nested  # nested(field, val) -> Thrift bytes of the JSON val as field.type

    def write_string_value(self, f: T.FieldDescriptor, val: str, enc: int) -> bytes:
        """writeStringValue conv/j2t/impl.go:107-151."""
        o = self.opts
        if val == "":
            if not o.WriteRequireField and f.required == T.REQUIRED:
                raise ConvError("ErrMissRequiredField", "required field '%s' not found" % f.name)
            if not o.WriteOptionalField and f.required == T.OPTIONAL:
                return b""
            if not o.WriteDefaultField and f.required == T.DEFAULT:
                return b""
            return field_begin(f) + write_default_or_empty(f)
        out = field_begin(f)
        if enc == ENCODING_THRIFT_BINARY:
            return out + val.encode("utf-8", "surrogateescape")
        if enc == ENCODING_TEXT or not _is_complex(f.type) or not is_json_string(val):
            try:
                return out + decode_text(val, f.type, o.DisallowUnknownField, not o.NoBase64Binary)
            except ValueError as e:
                raise ConvError("ErrConvert", "failed to write field '%s' value" % f.name, e)
        if enc == ENCODING_JSON:
            if self.nested is None:
                raise ConvError("ErrConvert", "failed to convert value of field '%s'" % f.name)
            return out + self.nested(f, val)
        raise ConvError("ErrConvert", "unsupported http-mapping encoding %d for '%s'" % (enc, f.name))

    def handle_http_mappings(self, req: Optional[HTTPRequest], sd: T.StructDescriptor,
                             nobody: bool) -> Tuple[bytes, int, Dict[int, bool]]:
        """handleHttpMappings conv/j2t/impl.go:243-292 for one struct: the
        mapped fields' bytes, the mask (by field index in id order, the
        descriptor blob's order) of the fields marked written
        (reqs.Set(id, Optional)), and the ids set back to Required
        (ReadHttpValueFallback: read them from the body)."""
        if req is None:
            raise ConvError("ErrInvalidParam", "http request is nil")
        order = {f.id: k for k, f in enumerate(sorted(sd.fields, key=lambda f: f.id))}
        out = b""
        mask = 0
        required_again: Dict[int, bool] = {}
        for f in sd.hms:
            ok, val, enc = False, "", ENCODING_TEXT
            for kind, value in f.http_mappings:
                v = mapping_request(kind, value, req, f)
                if v is not None:
                    enc, ok, val = mapping_encoding(kind), True, v
                    break
            if not ok:
                if nobody:
                    if f.required == T.REQUIRED and not self.opts.WriteRequireField:
                        raise ConvError("ErrNotFound", "not found http value of field %d:'%s'" % (f.id, f.name))
                    if not self.opts.WriteDefaultField and f.required == T.DEFAULT:
                        continue
                    if not self.opts.WriteOptionalField and f.required == T.OPTIONAL:
                        continue
                elif self.opts.ReadHttpValueFallback:
                    required_again[f.id] = True
                    continue
            mask |= 1 << order[f.id]
            out += self.write_string_value(f, val, enc)
        return out, mask, required_again

    def handle_unmatched_fields(self, req: Optional[HTTPRequest], sd: T.StructDescriptor, ids: List[int],
                                top: bool) -> bytes:
        """handleUnmatchedFields conv/j2t/impl_amd64.go:71-115, without the
        STOP (the caller writes it)."""
        if req is None:
            raise ConvError("ErrInvalidParam", "http request is nil")
        out = b""
        for fid in ids:
            f = sd.field_by_id(fid)
            if f is None:
                if self.opts.DisallowUnknownField:
                    raise ConvError("ErrConvert", "unknown field id %d" % fid)
                continue
            if f.is_request_base:
                continue
            val, enc = "", ENCODING_TEXT
            if self.opts.TracebackRequredOrRootFields and (top or f.required == T.REQUIRED):
                val, _, enc = try_get_value_from_http(req, f.alias)
            out += self.write_string_value(f, val, enc)
        return out

    def empty_body(self, req: Optional[HTTPRequest], sd: T.StructDescriptor) -> bytes:
        """The empty-body branch of BinaryConv.do conv/j2t/impl.go:52-82 with
        EnableHttpMapping and a request: mapped fields (nobody), then the
        required fields traced back on the request (HandleRequires with
        ReadHttpValueFallback), then STOP."""
        out = b""
        written = set()
        if sd.hms:
            b, mask, _ = self.handle_http_mappings(req, sd, True)
            out += b
            order = sorted(sd.fields, key=lambda f: f.id)
            written = {order[k].id for k in range(len(order)) if (mask >> k) & 1}
        fb = self.opts.ReadHttpValueFallback
        # RequiresBitmap.HandleRequires thrift/utils.go:149-176 over the bits
        # left set (required/default fields the mapping pass did not write)
        for f in sorted(sd.fields, key=lambda f: f.id):
            if f.id in written or not sd.requires.get(f.id, False):
                continue
            if f.required == T.REQUIRED and not fb:
                raise ConvError("ErrWrite", "failed to write required field",
                                ConvError("ErrMissRequiredField",
                                          "miss required field '%s' of struct '%s'" % (f.name, sd.name)))
            if (f.required == T.DEFAULT and not fb) or (f.required == T.OPTIONAL and not fb and f.default_value is None):
                continue
            val, _, enc = try_get_value_from_http(req, f.alias)
            out += self.write_string_value(f, val, enc)
        return out + b"\x00"


# ---------------------------------------------------------------- base.Base
class Base:
    """base.Base (kitex base.thrift, used by EnableThriftBase):
    1: string LogID, 2: string Caller, 3: string Addr, 4: string Client,
    5: optional TrafficEnv TrafficEnv {1: bool Open, 2: string Env},
    6: optional map<string, string> Extra."""

    def __init__(self, LogID="", Caller="", Addr="", Client="", TrafficEnv=None, Extra=None):
        self.LogID, self.Caller, self.Addr, self.Client = LogID, Caller, Addr, Client
        self.TrafficEnv = TrafficEnv  # None or (open: bool, env: str)
        self.Extra = Extra            # None or dict

    @staticmethod
    def from_json(obj) -> "Base":
        te = obj.get("TrafficEnv")
        return Base(obj.get("LogID", ""), obj.get("Caller", ""), obj.get("Addr", ""), obj.get("Client", ""),
                    (bool(te.get("Open", False)), te.get("Env", "")) if isinstance(te, dict) else None,
                    dict(obj["Extra"]) if isinstance(obj.get("Extra"), dict) else None)

    def thrift(self) -> bytes:
        """FastWrite: fields in id order, then STOP."""
        def s(fid, v):
            b = v.encode()
            return bytes([T.STRING]) + _st.pack(">hI", fid, len(b)) + b
        out = s(1, self.LogID) + s(2, self.Caller) + s(3, self.Addr) + s(4, self.Client)
        if self.TrafficEnv is not None:
            o, e = self.TrafficEnv
            eb = e.encode()
            out += bytes([T.STRUCT]) + _st.pack(">h", 5) + bytes([T.BOOL]) + _st.pack(">h", 1) + bytes([1 if o else 0])
            out += bytes([T.STRING]) + _st.pack(">hI", 2, len(eb)) + eb + b"\x00"
        if self.Extra is not None:
            out += bytes([T.MAP]) + _st.pack(">h", 6) + bytes([T.STRING, T.STRING]) + _st.pack(">I", len(self.Extra))
            for k, v in self.Extra.items():
                kb, vb = k.encode(), v.encode()
                out += _st.pack(">I", len(kb)) + kb + _st.pack(">I", len(vb)) + vb
        return out + b"\x00"


def write_request_base(base: Optional[Base], field: T.FieldDescriptor, src: bytes, merge) -> Tuple[bytes, bool]:
    """writeRequestBaseToThrift conv/j2t/impl.go:155-193: the Base field's
    bytes (field header + Base) and whether the body's own Base must be
    skipped (F_NO_WRITE_BASE: it was merged into the context's)."""
    if base is None:
        return b"", False
    no_write = False
    if src and merge is not None:
        members = _top_level_members(src)
        if members is not None and field.alias in members:
            a, b = members[field.alias]
            try:
                obj = _json.loads(src.decode("utf-8", "surrogateescape")[a:b])
                if isinstance(obj, dict):
                    base = merge(Base.from_json(obj), base)
            except ValueError:
                pass
            no_write = True
    return field_begin(field) + base.thrift(), no_write
