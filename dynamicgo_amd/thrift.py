"""Runtime Thrift type descriptors, a Thrift-IDL front end, and the flattener
that turns a descriptor graph into the position-independent ``dg_desc v1``
blob (include/dgj2t_desc.h) consumed by the HIP kernels.

Mirrors the reference's descriptor model:
  TypeDescriptor / StructDescriptor / FieldDescriptor  thrift/descriptor.go:119-267
  RequiresBitmap                                       thrift/utils.go:30-91
  IDL -> descriptor (parseType, convertRequireness,    thrift/idl.go:589-825
  makeDefaultValue, builtins)                          thrift/idl.go:834-955, 540-551
  field-name map (alias + name, last Set wins)         internal/util/fieldmap.go:50-62

This is host-side descriptor construction (init-time), not the
hot path. The IDL front end covers the subset the reference's testdata uses:
include, namespace, typedef, enum, const, struct/union/exception, service;
annotations go.tag json, api.key, api.js_conv, the api.* HTTP mappings, the
agw.* ones of InitAGWAnnos and registered value mappings.
"""
from __future__ import annotations

import os
import re
import struct as _st
from dataclasses import dataclass, field as _dcfield
from typing import Dict, List, Optional, Tuple

# ---- Thrift wire types (reference native/thrift.h:45-63, thrift/type.go) ----
STOP, VOID, BOOL, BYTE, I08, DOUBLE, I16, I32, I64, STRING, STRUCT, MAP, SET, LIST = (
    0, 1, 2, 3, 3, 4, 6, 8, 10, 11, 12, 13, 14, 15)
TYPE_NAMES = {BOOL: "BOOL", BYTE: "BYTE", DOUBLE: "DOUBLE", I16: "I16", I32: "I32",
              I64: "I64", STRING: "STRING", STRUCT: "STRUCT", MAP: "MAP", SET: "SET",
              LIST: "LIST", STOP: "STOP", VOID: "VOID"}

# ---- requireness (reference native/map.h:79-81, thrift/descriptor.go) ----
OPTIONAL, DEFAULT, REQUIRED = 0, 1, 2

VM_NONE = 0
VM_JSCONV = 101  # internal/types/types.go:445
VM_BODY_DYNAMIC = 257  # thrift/annotation/value_mapping.go:51

HTTP_MAPPING_KEYS = ("api.query", "api.path", "api.header", "api.cookie", "api.body",
                     "api.http_code", "api.raw_body", "api.form", "api.raw_uri",
                     "api.no_body_struct")  # thrift/annotation/register.go:28-37
ANNO_DEPRECATED = "dynamicgo.deprecated"  # AnnoKeyDynamicGoDeprecated, thrift/annotation.go:248


class TypeDescriptor:
    """thrift.TypeDescriptor (thrift/descriptor.go:119-125)."""

    __slots__ = ("type", "name", "key", "elem", "struct")

    def __init__(self, type: int, name: str, key=None, elem=None, struct=None):
        self.type = type
        self.name = name
        self.key = key
        self.elem = elem
        self.struct = struct

    def is_binary(self) -> bool:
        # native/thrift.c:1139 memeq(dc->name.buf, "binary", 6)
        return self.type == STRING and self.name[:6] == "binary"

    def __repr__(self):
        return f"TypeDescriptor({TYPE_NAMES.get(self.type, self.type)}, {self.name!r})"


@dataclass(eq=False)
class FieldDescriptor:
    """thrift.FieldDescriptor (thrift/descriptor.go:253-267)."""
    id: int
    name: str
    type: TypeDescriptor
    required: int = DEFAULT
    alias: Optional[str] = None
    vm: int = VM_NONE  # value-mapping annotation type; VM_JSCONV for api.js_conv
    default_value: Optional[bytes] = None  # IDL default as Thrift binary bytes
    is_request_base: bool = False
    is_response_base: bool = False
    http_mappings: List[Tuple[str, str]] = _dcfield(default_factory=list)  # (annotation key, value), IDL order
    value_mapping: Optional["ValueMapping"] = None  # FieldDescriptor.ValueMapping() (thrift/descriptor.go:318-321)

    def __post_init__(self):
        if self.alias is None:
            self.alias = self.name


class ValueMappingError(Exception):
    """An error a ValueMapping.write returns (wrapped by the caller as
    meta.ErrConvert "failed to convert field '<name>' value")."""


class ValueMapping:
    """thrift.ValueMapping (thrift/annotation.go): the non-inline value
    mappings the Go host runs on ERR_VM_END (handleValueMapping,
    conv/j2t/impl_amd64.go:117-155). ``write`` gets the field and the value's
    raw JSON text and returns the Thrift bytes BinaryProtocol would append
    after the field header (raise ValueMappingError to fail the message)."""

    def write(self, field: "FieldDescriptor", src: bytes) -> bytes:
        raise NotImplementedError


class AgwBodyDynamic(ValueMapping):
    """agwBodyDynamic.Write (thrift/annotation/value_mapping.go:101-106): the
    value's JSON text as a Thrift binary. The GPU serves it inline for STRING
    fields; this host copy only runs for the cases it refuses."""

    def write(self, field, src: bytes) -> bytes:
        if field.type.type != STRING:
            raise ValueMappingError("body_dynamic only support STRING type")
        return _st.pack(">I", len(src)) + bytes(src)


class _InlineJSConv(ValueMapping):
    """api.js_conv: inline on the device (native/thrift.c:514-634); never
    called back."""

    def write(self, field, src: bytes) -> bytes:  # pragma: no cover - inline
        raise ValueMappingError("api.js_conv is inline")


# annotation key -> (value-mapping type, ValueMapping) (thrift/annotation/register.go:42)
_VALUE_MAPPINGS: Dict[str, Tuple[int, ValueMapping]] = {"api.js_conv": (VM_JSCONV, _InlineJSConv())}
# key-mapping annotations (register.go:45): the field's JSON alias
_KEY_MAPPINGS = {"api.key"}
# agw.source / janus.source (sourceMapper, thrift/annotation/anno_mapping.go:
# 92-136), registered by init_agw_annos: source value -> HTTP mapping kind
_SOURCE_KEYS: set = set()
_SOURCE_KINDS = {"query": "api.query", "header": "api.header", "body": "api.body", "cookie": "api.cookie",
                 "post": "api.form", "path": "api.path", "raw_uri": "api.raw_uri", "raw_body": "api.raw_body",
                 "not_body_struct": "api.no_body_struct"}


def register_value_mapping(key: str, vm_type: int, mapping: ValueMapping):
    """thrift.RegisterAnnotation of a value-mapping annotation
    (thrift/annotation.go, e.g. value_mapping_test.go:46-48): fields annotated
    with `key` get value-mapping type `vm_type` (> 255: served by the host
    through `mapping` on ERR_VM_END)."""
    if not 0 < vm_type < 65536:
        raise ValueError("value-mapping type out of range")
    _VALUE_MAPPINGS[key] = (vm_type, mapping)


def init_agw_annos():
    """annotation.InitAGWAnnos (thrift/annotation/register.go:56-66), the
    parts j2t reads: agw.js_conv, agw.body_dynamic and agw.key."""
    _VALUE_MAPPINGS["agw.js_conv"] = (VM_JSCONV, _InlineJSConv())
    _VALUE_MAPPINGS["agw.body_dynamic"] = (VM_BODY_DYNAMIC, AgwBodyDynamic())
    _KEY_MAPPINGS.add("agw.key")
    _SOURCE_KEYS.update(("agw.source", "janus.source"))


class StructDescriptor:
    """thrift.StructDescriptor (thrift/descriptor.go:168-176).

    ``requires`` is the RequiresBitmap over field IDs; ``names`` is the
    field-name map (alias and name keys, last Set wins).
    """

    def __init__(self, name: str):
        self.name = name
        self.fields: List[FieldDescriptor] = []
        self.ids: Dict[int, FieldDescriptor] = {}
        self.names: Dict[str, FieldDescriptor] = {}
        self.requires: Dict[int, bool] = {}
        self.hms: List[FieldDescriptor] = []

    def add_field(self, f: FieldDescriptor, set_optional_bitmap: bool = False,
                  map_field_way: str = "both"):
        """thrift/idl.go:775-786 + convertRequireness thrift/idl.go:795-825."""
        self.fields.append(f)
        self.ids[f.id] = f
        if f.required == DEFAULT:
            req = REQUIRED if set_optional_bitmap else DEFAULT
        elif f.required == OPTIONAL:
            req = DEFAULT if set_optional_bitmap else OPTIONAL
        else:
            req = REQUIRED
        if f.is_request_base or f.is_response_base:
            req = OPTIONAL
        self.requires[f.id] = req != OPTIONAL
        if map_field_way == "alias":
            self.names[f.alias] = f
        elif map_field_way == "name":
            self.names[f.name] = f
        else:
            self.names[f.alias] = f
            self.names[f.name] = f
        if f.http_mappings:
            self.hms.append(f)
        return f

    def field_by_id(self, fid: int) -> Optional[FieldDescriptor]:
        return self.ids.get(fid)

    def requires_bitmap(self) -> List[int]:
        """The RequiresBitmap words (thrift/utils.go:45-79): bit id%64 of word
        id//64, set for Required/Default, clear for Optional; max id//64+1 words."""
        words = [0] * (max(self.requires, default=0) // 64 + 1)
        for fid, on in self.requires.items():
            if on:
                words[fid // 64] |= 1 << (fid % 64)
        return words

    def requires_is_set(self, fid: int) -> bool:
        """RequiresBitmap.IsSet (thrift/utils.go:64-71), out of range raises."""
        w = self.requires_bitmap()
        if fid // 64 >= len(w):
            raise IndexError("bitmap id out of range")
        return bool(w[fid // 64] >> (fid % 64) & 1)


# ---- builtins (thrift/idl.go:540-551) ----
def builtin(name: str) -> TypeDescriptor:
    t = {"bool": BOOL, "byte": BYTE, "i8": BYTE, "i16": I16, "i32": I32, "i64": I64,
         "double": DOUBLE, "string": STRING, "binary": STRING}[name]
    return TypeDescriptor(t, name)


def list_of(elem: TypeDescriptor) -> TypeDescriptor:
    return TypeDescriptor(LIST, "list", elem=elem)


def set_of(elem: TypeDescriptor) -> TypeDescriptor:
    return TypeDescriptor(SET, "set", elem=elem)


def map_of(key: TypeDescriptor, elem: TypeDescriptor) -> TypeDescriptor:
    return TypeDescriptor(MAP, "map", key=key, elem=elem)


def struct_type(name: str, fields=(), set_optional_bitmap=False) -> TypeDescriptor:
    """Build a STRUCT TypeDescriptor from FieldDescriptors (or tuples)."""
    sd = StructDescriptor(name)
    td = TypeDescriptor(STRUCT, name, struct=sd)
    for f in fields:
        if isinstance(f, tuple):
            f = FieldDescriptor(*f)
        sd.add_field(f, set_optional_bitmap=set_optional_bitmap)
    return td


# ---- Thrift binary encoding of IDL default values (thrift/idl.go:834-955) ----
def encode_default(t: TypeDescriptor, value) -> Optional[bytes]:
    if t.type == BOOL:
        return b"\x01" if value else b"\x00"
    if t.type == BYTE:
        return _st.pack(">b", ((int(value) + 128) & 0xff) - 128)
    if t.type == I16:
        return _st.pack(">h", ((int(value) + 2**15) & 0xffff) - 2**15)
    if t.type == I32:
        return _st.pack(">i", ((int(value) + 2**31) & 0xffffffff) - 2**31)
    if t.type == I64:
        return _st.pack(">q", ((int(value) + 2**63) & (2**64 - 1)) - 2**63)
    if t.type == DOUBLE:
        return _st.pack(">d", float(value))
    if t.type == STRING:
        b = value.encode() if isinstance(value, str) else bytes(value)
        return _st.pack(">I", len(b)) + b
    return None


# ============================================================================
# flattening: descriptor graph -> dg_desc v1 blob (include/dgj2t_desc.h)
# ============================================================================
DG_DESC_MAGIC = 0x31444744
DG_NONE = 0xFFFFFFFF
HDR_FMT = "<16I"
TYPE_FMT = "<BBHIII"
STRUCT_FMT = "<8I"
FIELD_FMT = "<HbBHHIIII"
NAME_FMT = "<4I"


def name_hash(key: bytes) -> int:
    """DG_NAME_HASH_STEP in include/dgj2t_desc.h."""
    h = 5381
    for b in key:
        h = (((h << 5) + h) & 0xFFFFFFFF) ^ b
    return h


class FlatDescriptor:
    """A flattened descriptor blob plus the index of the root type."""

    def __init__(self, blob: bytes, root_type: int, types: List[TypeDescriptor]):
        self.blob = blob
        self.root_type = root_type
        self.types = types

    def __len__(self):
        return len(self.blob)


def _align8(b: bytearray):
    while len(b) % 8:
        b.append(0)


def flatten(root: TypeDescriptor) -> FlatDescriptor:
    """Serialize the (possibly cyclic) graph reachable from ``root``."""
    types: List[TypeDescriptor] = []
    tindex: Dict[int, int] = {}
    structs: List[StructDescriptor] = []
    sindex: Dict[int, int] = {}

    def visit(t: TypeDescriptor) -> int:
        k = id(t)
        if k in tindex:
            return tindex[k]
        tindex[k] = len(types)
        types.append(t)
        if t.key is not None:
            visit(t.key)
        if t.elem is not None:
            visit(t.elem)
        if t.struct is not None:
            sk = id(t.struct)
            if sk not in sindex:
                sindex[sk] = len(structs)
                structs.append(t.struct)
                for f in sorted(t.struct.fields, key=lambda f: f.id):
                    visit(f.type)
        return tindex[k]

    root_idx = visit(root)

    pool = bytearray()
    pool_index: Dict[bytes, int] = {}

    def pool_put(b: bytes) -> int:
        if b in pool_index:
            return pool_index[b]
        off = len(pool)
        pool.extend(b)
        pool_index[b] = off
        return off

    key_index: Dict[bytes, int] = {}

    def pool_key(b: bytes) -> int:
        # keys: 8-aligned and zero-padded so the fast path compares whole words
        if b in key_index:
            return key_index[b]
        while len(pool) % 8:
            pool.append(0)
        off = len(pool)
        pool.extend(b)
        while len(pool) % 8 or len(pool) == off:
            pool.append(0)
        key_index[b] = off
        return off

    type_rows = []
    for t in types:
        flags = 1 if t.is_binary() else 0
        type_rows.append(_st.pack(
            TYPE_FMT, t.type, flags, 0,
            tindex[id(t.key)] if t.key is not None else DG_NONE,
            tindex[id(t.elem)] if t.elem is not None else DG_NONE,
            sindex[id(t.struct)] if t.struct is not None else DG_NONE))

    field_rows, name_rows, req_words, struct_rows = [], [], [], []
    field_objs: List[FieldDescriptor] = []  # blob order (t2j side table)
    for sd in structs:
        fields = sorted(sd.fields, key=lambda f: f.id)
        # a field id may be Set twice in the IDL (ids.Set overwrites); keep last
        dedup: Dict[int, FieldDescriptor] = {}
        for f in fields:
            dedup[f.id] = sd.ids[f.id]
        fields = [dedup[k] for k in sorted(dedup)]
        fbegin = len(field_rows)
        findex = {id(f): fbegin + i for i, f in enumerate(fields)}
        for f in fields:
            field_objs.append(f)
            fl = (1 if f.is_request_base else 0) | (2 if f.http_mappings else 0) | (16 if f.is_response_base else 0)
            if sd.names.get(f.alias) is f:
                fl |= 4  # DG_FF_ALIAS_SELF
            if b'"' not in f.alias.encode() and b"\\" not in f.alias.encode():
                fl |= 8  # DG_FF_KEY_PLAIN
            if f.default_value is not None:
                doff, dlen = pool_put(bytes(f.default_value)), len(f.default_value)
            else:
                doff, dlen = 0, DG_NONE
            ak = f.alias.encode()
            field_rows.append(_st.pack(FIELD_FMT, f.id, f.required, fl, f.vm, len(ak),
                                       tindex[id(f.type)], doff, dlen, pool_key(ak)))
        # requires bits by field index
        nw = max(1, (len(fields) + 63) // 64)
        words = [0] * nw
        for i, f in enumerate(fields):
            if sd.requires.get(f.id, False):
                words[i // 64] |= 1 << (i % 64)
        rbegin = len(req_words)
        req_words.extend(words)
        # name table (open addressing, load <= 0.5)
        size = 2
        while size < 2 * max(1, len(sd.names)):
            size *= 2
        slots = [None] * size
        for key, f in sd.names.items():
            kb = key.encode()
            h = name_hash(kb)
            j = h & (size - 1)
            while slots[j] is not None:
                j = (j + 1) & (size - 1)
            slots[j] = (h, pool_key(kb), len(kb), findex[id(sd.ids[f.id])])
        nbegin = len(name_rows)
        for s in slots:
            name_rows.append(_st.pack(NAME_FMT, *(s if s else (0, 0, 0, DG_NONE))))
        struct_rows.append(_st.pack(STRUCT_FMT, fbegin, len(fields), nbegin, size - 1,
                                    rbegin, nw, 1 if sd.hms else 0, 0))

    body = bytearray(64)
    offs = []
    for rows in (type_rows, struct_rows, field_rows, name_rows):
        _align8(body)
        offs.append(len(body))
        for r in rows:
            body.extend(r)
    _align8(body)
    offs.append(len(body))
    for w in req_words:
        body.extend(_st.pack("<Q", w))
    _align8(body)
    offs.append(len(body))
    body.extend(pool)
    _align8(body)
    hdr = _st.pack(HDR_FMT, DG_DESC_MAGIC, 2, len(body), root_idx,
                   len(type_rows), offs[0], len(struct_rows), offs[1],
                   len(field_rows), offs[2], len(name_rows), offs[3],
                   len(req_words), offs[4], len(pool), offs[5])
    body[:64] = hdr
    fd = FlatDescriptor(bytes(body), root_idx, types)
    fd.fields = field_objs
    fd.structs = structs  # StructDescriptors in blob order (the HTTP-mapping table's slots)
    return fd


def json_quote(b: bytes) -> bytes:
    r"""The reference's native quote() with flags 0 (native/parsing.c:28-63,
    _SingleQuoteTab): '"' and '\\' backslashed, \t \n \r short, every other
    byte < 0x20 as \u00xx; no HTML escaping, no UTF-8 check."""
    out = bytearray()
    for c in b:
        if c == 0x22:
            out += b'\\"'
        elif c == 0x5C:
            out += b"\\\\"
        elif c == 0x09:
            out += b"\\t"
        elif c == 0x0A:
            out += b"\\n"
        elif c == 0x0D:
            out += b"\\r"
        elif c < 0x20:
            out += b"\\u%04x" % c
        else:
            out.append(c)
    return bytes(out)


DG_T2J_MAGIC = 0x32544744


def flatten_t2j(fd: FlatDescriptor) -> bytes:
    """The t2j side table of a flattened descriptor (include/dgj2t_desc.h
    dg_t2j_*): per field, json.EncodeString(alias) + ':' and
    EncodeString(name) + ':' (conv/t2j/impl.go:150-152, 431-433), and the raw
    alias / name bytes."""
    pool = bytearray()

    def put(b: bytes):
        off = len(pool)
        pool.extend(b)
        while len(pool) % 8:
            pool.append(0)
        return off, len(b)

    rows = []
    for f in fd.fields:
        a, n = f.alias.encode(), f.name.encode()
        rows.append(_st.pack("<8I", *put(b'"' + json_quote(a) + b'":'), *put(b'"' + json_quote(n) + b'":'),
                             *put(a), *put(n)))
    off_fields = 32
    off_pool = off_fields + 32 * len(rows)
    body = _st.pack("<8I", DG_T2J_MAGIC, 1, off_pool + len(pool) + 16, len(rows), off_fields, len(pool), off_pool, 0)
    return body + b"".join(rows) + bytes(pool) + bytes(16)


# ============================================================================
# Thrift IDL front end (subset of thriftgo's grammar)
# ============================================================================
_TOKEN_RE = re.compile(r"""
    (?P<ws>\s+|//[^\n]*|\#[^\n]*|/\*.*?\*/)
  | (?P<str>"(?:[^"\\]|\\.)*"|'(?:[^'\\]|\\.)*')
  | (?P<num>[+-]?(?:0x[0-9a-fA-F]+|\d+\.\d*(?:[eE][+-]?\d+)?|\d+[eE][+-]?\d+|\.\d+(?:[eE][+-]?\d+)?|\d+))
  | (?P<id>[A-Za-z_][A-Za-z0-9_.]*)
  | (?P<sym>[{}()<>\[\]=:;,*])
""", re.S | re.X)


def _tokenize(src: str):
    out, i = [], 0
    while i < len(src):
        m = _TOKEN_RE.match(src, i)
        if not m:
            raise SyntaxError(f"bad IDL char {src[i]!r} at {i}")
        i = m.end()
        k = m.lastgroup
        if k == "ws":
            continue
        out.append((k, m.group(k)))
    return out


def _unquote_lit(s: str) -> str:
    body = s[1:-1]
    return re.sub(r"\\(.)", lambda m: {"n": "\n", "t": "\t", "r": "\r"}.get(m.group(1), m.group(1)), body)


@dataclass
class _PType:
    name: str
    key: Optional["_PType"] = None
    val: Optional["_PType"] = None


@dataclass
class _PField:
    id: int
    req: str
    type: _PType
    name: str
    default: object
    annos: List[Tuple[str, str]]


class _Parser:
    def __init__(self, toks):
        self.t = toks
        self.i = 0

    def peek(self, k=0):
        j = self.i + k
        return self.t[j] if j < len(self.t) else (None, None)

    def next(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def accept(self, v):
        if self.peek()[1] == v:
            self.i += 1
            return True
        return False

    def expect(self, v):
        k, x = self.next()
        if x != v:
            raise SyntaxError(f"expected {v!r} got {x!r}")

    def sep(self):
        if self.peek()[1] in (",", ";"):
            self.i += 1

    def ident(self):
        k, x = self.next()
        if k != "id":
            raise SyntaxError(f"expected identifier got {x!r}")
        return x

    def annotations(self):
        annos = []
        if self.accept("("):
            while not self.accept(")"):
                k = self.ident()
                v = ""
                if self.accept("="):
                    v = _unquote_lit(self.next()[1])
                annos.append((k, v))
                self.sep()
        return annos

    def ptype(self) -> _PType:
        n = self.ident()
        if n in ("list", "set"):
            self.expect("<")
            v = self.ptype()
            self.expect(">")
            t = _PType(n, val=v)
        elif n == "map":
            self.expect("<")
            k = self.ptype()
            self.expect(",")
            v = self.ptype()
            self.expect(">")
            t = _PType(n, key=k, val=v)
        else:
            t = _PType(n)
        self.annotations()
        return t

    def const_value(self):
        k, x = self.peek()
        if x == "[":
            self.next()
            out = []
            while not self.accept("]"):
                out.append(self.const_value())
                self.sep()
            return ("list", out)
        if x == "{":
            self.next()
            out = []
            while not self.accept("}"):
                kk = self.const_value()
                self.expect(":")
                out.append((kk, self.const_value()))
                self.sep()
            return ("map", out)
        self.next()
        if k == "num":
            if re.fullmatch(r"[+-]?(0x[0-9a-fA-F]+|\d+)", x):
                return ("int", int(x, 0))
            return ("double", float(x))
        if k == "str":
            return ("lit", _unquote_lit(x))
        return ("ident", x)

    def fields(self):
        out = []
        self.expect("{")
        while not self.accept("}"):
            fid = None
            if self.peek()[0] == "num" and self.peek(1)[1] == ":":
                fid = int(self.next()[1], 0)
                self.expect(":")
            req = "default"
            if self.peek()[1] in ("required", "optional"):
                req = self.next()[1]
            t = self.ptype()
            name = self.ident()
            dv = None
            if self.accept("="):
                dv = self.const_value()
            annos = self.annotations()
            self.sep()
            out.append(_PField(fid if fid is not None else -len(out) - 1, req, t, name, dv, annos))
        return out


class IDLFile:
    def __init__(self, path: str, src: str, includes: Dict[str, str]):
        self.path = path
        self.includes: Dict[str, "IDLFile"] = {}
        self.typedefs: Dict[str, _PType] = {}
        self.enums: Dict[str, Dict[str, int]] = {}
        self.consts: Dict[str, object] = {}
        self.structs: Dict[str, List[_PField]] = {}
        self.services: Dict[str, Dict[str, Tuple[_PType, List[_PField]]]] = {}
        p = _Parser(_tokenize(src))
        while p.peek()[0] is not None:
            kw = p.ident()
            if kw in ("include", "cpp_include"):
                inc = _unquote_lit(p.next()[1])
                if kw == "include":
                    ipath = os.path.normpath(os.path.join(os.path.dirname(path), inc))
                    isrc = includes.get(ipath)
                    if isrc is None:
                        isrc = includes.get(inc)
                    if isrc is None:
                        with open(ipath) as fh:
                            isrc = fh.read()
                    key = os.path.splitext(os.path.basename(inc))[0]
                    self.includes[key] = IDLFile(ipath, isrc, includes)
            elif kw == "namespace":
                p.ident()
                p.ident()
                p.annotations()
            elif kw == "typedef":
                t = p.ptype()
                self.typedefs[p.ident()] = t
                p.annotations()
            elif kw == "enum":
                name = p.ident()
                p.expect("{")
                vals, cur = {}, 0
                while not p.accept("}"):
                    n = p.ident()
                    if p.accept("="):
                        cur = int(p.next()[1], 0)
                    vals[n] = cur
                    cur += 1
                    p.annotations()
                    p.sep()
                self.enums[name] = vals
                p.annotations()
            elif kw == "const":
                p.ptype()
                n = p.ident()
                p.expect("=")
                self.consts[n] = p.const_value()
                p.sep()
            elif kw in ("struct", "union", "exception"):
                name = p.ident()
                self.structs[name] = p.fields()
                p.annotations()
            elif kw == "service":
                name = p.ident()
                if p.accept("extends"):
                    p.ident()
                p.expect("{")
                funcs = {}
                while not p.accept("}"):
                    p.accept("oneway")
                    rt = p.ptype()
                    fname = p.ident()
                    p.expect("(")
                    args = []
                    while not p.accept(")"):
                        fid = int(p.next()[1], 0)
                        p.expect(":")
                        req = "default"
                        if p.peek()[1] in ("required", "optional"):
                            req = p.next()[1]
                        t = p.ptype()
                        an = p.ident()
                        annos = p.annotations()
                        p.sep()
                        args.append(_PField(fid, req, t, an, None, annos))
                    throws = []
                    if p.accept("throws"):
                        p.expect("(")
                        while not p.accept(")"):
                            fid = int(p.next()[1], 0)
                            p.expect(":")
                            if p.peek()[1] in ("required", "optional"):
                                p.next()
                            t = p.ptype()
                            throws.append(_PField(fid, "default", t, p.ident(), None, p.annotations()))
                            p.sep()
                    p.annotations()
                    p.sep()
                    funcs[fname] = (rt, args, throws)
                self.services[name] = funcs
                p.annotations()
            else:
                raise SyntaxError(f"unsupported IDL keyword {kw!r}")


@dataclass
class Options:
    """thrift.Options subset (thrift/idl.go:51-107)."""
    use_default_value: bool = False
    set_optional_bitmap: bool = False
    parse_enum_as_int64: bool = False
    map_field_way: str = "both"  # "alias" | "name" | "both"
    enable_thrift_base: bool = False


class _Compiler:
    def __init__(self, root: IDLFile, opts: Options):
        self.root = root
        self.opts = opts

    def resolve(self, f: IDLFile, name: str):
        """An include's prefix is its file name less ".thrift", dots included
        ("deep/deep.ref.thrift" -> "deep.ref."): the longest matching prefix wins."""
        best = None
        for pkg in f.includes:
            if name.startswith(pkg + ".") and (best is None or len(pkg) > len(best)):
                best = pkg
        if best is not None:
            return f.includes[best], name[len(best) + 1:]
        return f, name

    def const_default(self, f: IDLFile, t: TypeDescriptor, cv) -> Optional[bytes]:
        """makeDefaultValue (thrift/idl.go:834-955)."""
        if cv is None:
            return None
        kind, v = cv
        if kind == "int":
            return encode_default(t, v) if t.type in (BYTE, I16, I32, I64) else None
        if kind == "double":
            return encode_default(t, v) if t.type == DOUBLE else None
        if kind == "lit":
            return encode_default(t, v) if t.type == STRING else None
        if kind == "ident":
            if t.type == BOOL and v.lower() in ("true", "false"):
                return b"\x01" if v.lower() == "true" else b"\x00"
            ff, name = self.resolve(f, v)
            if name in ff.consts:
                return self.const_default(ff, t, ff.consts[name])
            if "." in name:
                en, val = name.rsplit(".", 1)
                ef, en = self.resolve(ff, en)
                if en in ef.enums and val in ef.enums[en] and t.type in (BYTE, I16, I32, I64):
                    return encode_default(t, ef.enums[en][val])
        return None

    def ptype(self, f: IDLFile, pt: _PType, cache, depth: int) -> TypeDescriptor:
        """parseType (thrift/idl.go:589-793)."""
        if pt.name in ("bool", "byte", "i8", "i16", "i32", "i64", "double", "string", "binary"):
            return builtin(pt.name)
        if pt.name in ("list", "set"):
            e = self.ptype(f, pt.val, cache, depth + 1)
            return list_of(e) if pt.name == "list" else set_of(e)
        if pt.name == "map":
            return map_of(self.ptype(f, pt.key, cache, depth + 1),
                          self.ptype(f, pt.val, cache, depth + 1))
        ck = (id(f), pt.name)
        if ck in cache:
            return cache[ck]
        ff, name = self.resolve(f, pt.name)
        if ff is not f:
            cache = {}
        if name in ff.typedefs:
            return self.ptype(ff, ff.typedefs[name], cache, depth + 1)
        if name in ff.enums:
            return builtin("i64" if self.opts.parse_enum_as_int64 else "i32")
        if name not in ff.structs:
            raise KeyError(f"missing type: {pt.name}")
        sd = StructDescriptor(pt.name)
        td = TypeDescriptor(STRUCT, pt.name, struct=sd)
        cache[ck] = td
        for pf in ff.structs[name]:
            if any(k == ANNO_DEPRECATED for k, _ in pf.annos):
                continue  # handleNativeFieldAnnotation (thrift/annotation.go:399-404): field dropped
            alias = pf.name
            vm = VM_NONE
            vmap = None
            hms = []
            sources = []
            for k, v in pf.annos:
                if k == "go.tag":
                    m = re.search(r'json:"([^"]*)"', v) or re.search(r"json:\\\"([^\\]*)\\\"", v)
                    if m:
                        alias = m.group(1).split(",")[0] or alias
                elif k in _KEY_MAPPINGS:
                    alias = v
                elif k in _VALUE_MAPPINGS:
                    vm, vmap = _VALUE_MAPPINGS[k]
                elif k in HTTP_MAPPING_KEYS:
                    hms.append((k, v))
                elif k in _SOURCE_KEYS:
                    sources.append(v)
            if sources:
                # decideNameCase (anno_mapping.go:138-163): api.key / agw.key, else
                # the field name (the agw.to_snake-style name cases are not restated)
                name = next((v for k, v in pf.annos if k in ("api.key", "agw.key") and v), pf.name)
                for v in sources:
                    kind = _SOURCE_KINDS.get(v.lower())
                    if kind is not None:
                        hms.append((kind, name))
            is_req_base = (self.opts.enable_thrift_base and pf.type.name == "base.Base" and depth == 0)
            is_resp_base = (self.opts.enable_thrift_base and pf.type.name == "base.BaseResp" and depth == 0)
            ftype = self.ptype(ff, pf.type, cache, depth + 1)
            dflt = self.const_default(ff, ftype, pf.default) if self.opts.use_default_value else None
            req = {"default": DEFAULT, "optional": OPTIONAL, "required": REQUIRED}[pf.req]
            sd.add_field(FieldDescriptor(pf.id, pf.name, ftype, req, alias, vm, dflt,
                                         is_req_base, is_resp_base, hms, vmap),
                         set_optional_bitmap=self.opts.set_optional_bitmap,
                         map_field_way=self.opts.map_field_way)
        return td


class FunctionDescriptor:
    def __init__(self, name, request: TypeDescriptor, response: Optional[TypeDescriptor]):
        self.name = name
        self._req = request
        self._resp = response

    def request(self) -> TypeDescriptor:
        return self._req

    def response(self) -> Optional[TypeDescriptor]:
        return self._resp


class ServiceDescriptor:
    def __init__(self, name: str, functions: Dict[str, FunctionDescriptor]):
        self.name = name
        self._functions = functions

    def functions(self) -> Dict[str, FunctionDescriptor]:
        return self._functions


def _parse_service(path: str, src: str, includes: Dict[str, str], opts: Options,
                   service: Optional[str] = None) -> ServiceDescriptor:
    root = IDLFile(path, src, includes or {})
    if not root.services:
        raise ValueError("no service in IDL")
    sname = service or list(root.services)[-1]
    comp = _Compiler(root, opts)
    funcs = {}
    for fname, (rt, args, throws) in root.services[sname].items():
        cache: dict = {}
        req_sd = StructDescriptor(fname + "_args")
        for a in args:
            req_sd.add_field(FieldDescriptor(a.id, a.name, comp.ptype(root, a.type, cache, 0)))
        req_td = TypeDescriptor(STRUCT, fname + "_args", struct=req_sd)
        resp_td = None
        if rt.name != "void":
            # parseResponse (thrift/idl.go:490-537): the result wrapper, the
            # response as field 0 with no name, the first thrown exception
            resp_sd = StructDescriptor(fname + "_result")
            resp_sd.add_field(FieldDescriptor(0, "", comp.ptype(root, rt, {}, 0), OPTIONAL, alias=""))
            if throws:
                e = throws[0]
                resp_sd.add_field(FieldDescriptor(e.id, e.name, comp.ptype(root, e.type, {}, 0), OPTIONAL))
            resp_td = TypeDescriptor(STRUCT, fname + "_result", struct=resp_sd)
        funcs[fname] = FunctionDescriptor(fname, req_td, resp_td)
    return ServiceDescriptor(sname, funcs)


def new_descriptor_from_path(path: str, opts: Optional[Options] = None, service=None) -> ServiceDescriptor:
    """thrift.Options.NewDescritorFromPath (thrift/idl.go:131)."""
    with open(path) as fh:
        return _parse_service(path, fh.read(), {}, opts or Options(), service)


def new_descriptor_from_content(path: str, content: str, includes=None,
                                opts: Optional[Options] = None, service=None) -> ServiceDescriptor:
    """thrift.Options.NewDescritorFromContent (thrift/idl.go:167)."""
    return _parse_service(path, content, includes or {}, opts or Options(), service)


def new_descriptor_by_name(path: str, content: str, name: str, includes=None,
                           opts: Optional[Options] = None) -> TypeDescriptor:
    """thrift.Options.NewDescriptorByName (thrift/idl.go:957): one named type."""
    root = IDLFile(path, content, includes or {})
    return _Compiler(root, opts or Options()).ptype(root, _PType(name), {}, 0)
