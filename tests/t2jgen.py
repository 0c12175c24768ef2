"""Random Thrift-binary inputs for the t2j parity tests: every wire type,
unknown fields (the skip path), recursion, js_conv fields, special strings and
doubles, and mutations for the error paths. Seeded; pure Python."""
import random
import struct

from dynamicgo_amd import thrift as T

BOOL, BYTE, DOUBLE, I16, I32, I64, STRING, STRUCT, MAP, SET, LIST = 2, 3, 4, 6, 8, 10, 11, 12, 13, 14, 15


def all_types_desc(with_default=False, alias_quirks=True):
    """A struct using every type the t2j path handles (and a recursive
    child), with required / default / optional fields and js_conv fields."""
    node_sd = T.StructDescriptor("Node")
    node = T.TypeDescriptor(STRUCT, "Node", struct=node_sd)
    node_sd.add_field(T.FieldDescriptor(1, "val", T.builtin("i32"), T.OPTIONAL))
    node_sd.add_field(T.FieldDescriptor(2, "next", node, T.OPTIONAL))
    node_sd.add_field(T.FieldDescriptor(3, "kids", T.list_of(node), T.OPTIONAL))
    inner = T.struct_type("Inner", [
        T.FieldDescriptor(1, "a", T.builtin("i64"), T.REQUIRED),
        T.FieldDescriptor(2, "b", T.builtin("string"), T.DEFAULT),
        T.FieldDescriptor(3, "c", T.list_of(T.builtin("double")), T.OPTIONAL),
    ])
    f = [
        T.FieldDescriptor(1, "bool_f", T.builtin("bool"), T.OPTIONAL),
        T.FieldDescriptor(2, "byte_f", T.builtin("byte"), T.OPTIONAL),
        T.FieldDescriptor(3, "i16_f", T.builtin("i16"), T.DEFAULT),
        T.FieldDescriptor(4, "i32_f", T.builtin("i32"), T.OPTIONAL),
        T.FieldDescriptor(5, "i64_f", T.builtin("i64"), T.OPTIONAL),
        T.FieldDescriptor(6, "dbl_f", T.builtin("double"), T.OPTIONAL),
        T.FieldDescriptor(7, "str_f", T.builtin("string"), T.OPTIONAL,
                          alias='q"uo\\teé\x01' if alias_quirks else None),
        T.FieldDescriptor(8, "bin_f", T.builtin("binary"), T.OPTIONAL),
        T.FieldDescriptor(9, "inner", inner, T.OPTIONAL),
        T.FieldDescriptor(10, "inners", T.list_of(inner), T.OPTIONAL),
        T.FieldDescriptor(11, "set_f", T.set_of(T.builtin("i64")), T.OPTIONAL),
        T.FieldDescriptor(12, "m_str", T.map_of(T.builtin("string"), T.list_of(T.builtin("i32"))), T.OPTIONAL),
        T.FieldDescriptor(13, "m_i8", T.map_of(T.builtin("byte"), T.builtin("bool")), T.OPTIONAL),
        T.FieldDescriptor(14, "m_i16", T.map_of(T.builtin("i16"), T.builtin("binary")), T.OPTIONAL),
        T.FieldDescriptor(15, "m_i32", T.map_of(T.builtin("i32"), inner), T.OPTIONAL),
        T.FieldDescriptor(16, "m_i64", T.map_of(T.builtin("i64"), T.map_of(T.builtin("string"), T.builtin("double"))),
                          T.OPTIONAL),
        T.FieldDescriptor(17, "node", node, T.OPTIONAL),
        T.FieldDescriptor(18, "req_s", T.builtin("string"), T.REQUIRED),
        T.FieldDescriptor(19, "def_l", T.list_of(T.builtin("string")), T.DEFAULT),
        T.FieldDescriptor(20, "def_m", T.map_of(T.builtin("string"), T.builtin("i64")), T.DEFAULT),
        T.FieldDescriptor(21, "def_st", inner, T.DEFAULT),
        T.FieldDescriptor(22, "def_d", T.builtin("double"), T.DEFAULT),
        T.FieldDescriptor(23, "def_b", T.builtin("bool"), T.DEFAULT),
        T.FieldDescriptor(24, "def_y", T.builtin("byte"), T.DEFAULT),
        T.FieldDescriptor(30, "vm_i64", T.builtin("i64"), T.OPTIONAL, vm=T.VM_JSCONV),
        T.FieldDescriptor(31, "vm_l32", T.list_of(T.builtin("i32")), T.OPTIONAL, vm=T.VM_JSCONV),
        T.FieldDescriptor(32, "vm_s", T.builtin("string"), T.OPTIONAL, vm=T.VM_JSCONV),
        T.FieldDescriptor(33, "vm_d", T.builtin("double"), T.OPTIONAL, vm=T.VM_JSCONV),
        T.FieldDescriptor(34, "vm_y", T.builtin("byte"), T.OPTIONAL, vm=T.VM_JSCONV),
        T.FieldDescriptor(35, "vm_l16", T.list_of(T.builtin("i16")), T.OPTIONAL, vm=T.VM_JSCONV),
        T.FieldDescriptor(32767, "max_id", T.builtin("i16"), T.OPTIONAL),
    ]
    if with_default:
        f.append(T.FieldDescriptor(40, "with_dflt", T.builtin("i32"), T.OPTIONAL,
                                   default_value=T.encode_default(T.builtin("i32"), 7)))
        f.append(T.FieldDescriptor(41, "d_str", T.builtin("string"), T.DEFAULT,
                                   default_value=T.encode_default(T.builtin("string"), 'q"\\x\u00e9')))
        f.append(T.FieldDescriptor(42, "d_dbl", T.builtin("double"), T.OPTIONAL,
                                   default_value=T.encode_default(T.builtin("double"), -1.25e-7)))
        f.append(T.FieldDescriptor(43, "d_bool", T.builtin("bool"), T.DEFAULT,
                                   default_value=T.encode_default(T.builtin("bool"), True)))
        f.append(T.FieldDescriptor(44, "d_i8", T.builtin("byte"), T.REQUIRED,
                                   default_value=T.encode_default(T.builtin("byte"), -3)))
        f.append(T.FieldDescriptor(45, "d_list", T.list_of(T.builtin("i32")), T.OPTIONAL,
                                   default_value=bytes([8, 0, 0, 0, 1, 0, 0, 0, 4])))  # container: NEEDS_HOST
    return T.struct_type("All", f)


def wide_desc(n=70):
    """A struct of n > 64 fields (the GPU leaves it to the host)."""
    return T.struct_type("Wide", [T.FieldDescriptor(i + 1, f"f{i}", T.builtin("i32"), T.OPTIONAL) for i in range(n)])


def chain_desc():
    sd = T.StructDescriptor("Chain")
    td = T.TypeDescriptor(STRUCT, "Chain", struct=sd)
    sd.add_field(T.FieldDescriptor(1, "v", T.builtin("i32"), T.OPTIONAL))
    sd.add_field(T.FieldDescriptor(2, "next", td, T.OPTIONAL))
    return td


def chain_thrift(depth):
    """Chain nested `depth` levels (depth containers)."""
    return (b"\x0c\x00\x02" * (depth - 1)) + b"\x08\x00\x01\x00\x00\x00\x07" + b"\x00" * depth


_SPECIAL = [b'"', b"\\", b"\n", b"\r", b"\t", b"\x00", b"\x01", b"\x1f", b"\x7f", b"/", b"<", b"&",
            "é".encode(), "中文".encode(), "😀".encode(), b"\xff", b"\xc3", b"\xe2\x80\xa8", b"\xe2\x80\xa9"]


def rbytes(rng, maxn=24):
    out = bytearray()
    for _ in range(rng.randrange(maxn + 1)):
        r = rng.random()
        if r < 0.7:
            out.append(rng.randrange(0x20, 0x7f))
        else:
            out += rng.choice(_SPECIAL)
    return bytes(out)


def rdouble(rng, nan_p=0.0):
    r = rng.random()
    if r < nan_p:
        return rng.choice([float("nan"), float("inf"), float("-inf")])
    r = rng.random()
    if r < 0.15:
        return float(rng.randrange(-10**6, 10**6))
    if r < 0.3:
        return rng.uniform(-1000, 1000)
    if r < 0.4:
        return rng.choice([0.0, -0.0, 1e21, 1e20, 123456789012345678901.0, 1e-7, 1e-6, 0.1, 5e-324,
                           2.2250738585072014e-308, 1.7976931348623157e308, 9007199254740993.0, 0.3])
    if r < 0.55:
        return rng.uniform(-1, 1) * 10.0 ** rng.randrange(-30, 30)
    while True:  # random bits: subnormals, huge and tiny exponents
        bits = rng.getrandbits(64)
        if (bits >> 52) & 0x7FF != 0x7FF:
            return struct.unpack("<d", struct.pack("<Q", bits))[0]


def rint(rng, bits):
    lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
    r = rng.random()
    if r < 0.2:
        return rng.choice([0, -1, 1, lo, hi, 10, 99, 100, -100])
    if r < 0.6:
        return rng.randrange(max(lo, -1000), min(hi, 1000) + 1)
    return rng.randrange(lo, hi + 1)


_PK = {BYTE: ">b", I16: ">h", I32: ">i", I64: ">q"}


def w_scalar(rng, t, out, nan_p):
    if t == BOOL:
        out.append(rng.choice([0, 1, 1, 2]))
    elif t in _PK:
        out += struct.pack(_PK[t], rint(rng, {BYTE: 8, I16: 16, I32: 32, I64: 64}[t]))
    elif t == DOUBLE:
        out += struct.pack(">d", rdouble(rng, nan_p))
    elif t == STRING:
        s = rbytes(rng)
        out += struct.pack(">i", len(s)) + s
    else:
        raise ValueError(t)


def w_any(rng, out, depth):
    """A value of a random wire type (for unknown fields); returns its type."""
    t = rng.choice([BOOL, BYTE, I16, I32, I64, DOUBLE, STRING, STRING, STRUCT, LIST, SET, MAP] if depth < 4
                   else [BOOL, I32, STRING])
    if t == STRUCT:
        for _ in range(rng.randrange(3)):
            pos = len(out)
            out += b"\x00\x00\x00"
            ft = w_any(rng, out, depth + 1)
            out[pos] = ft
            out[pos + 1:pos + 3] = struct.pack(">h", rng.randrange(1, 100))
        out.append(0)
    elif t in (LIST, SET):
        et = rng.choice([I32, STRING, STRUCT, LIST, DOUBLE])
        n = rng.randrange(4)
        out.append(et)
        out += struct.pack(">i", n)
        for _ in range(n):
            w_typed_any(rng, et, out, depth + 1)
    elif t == MAP:
        kt, vt = rng.choice([I32, STRING, I64]), rng.choice([I32, STRING, STRUCT, MAP, BOOL])
        n = rng.randrange(4)
        out += bytes([kt, vt]) + struct.pack(">i", n)
        for _ in range(n):
            w_typed_any(rng, kt, out, depth + 1)
            w_typed_any(rng, vt, out, depth + 1)
    else:
        w_scalar(rng, t, out, 0.0)
    return t


def w_typed_any(rng, t, out, depth):
    if t in (STRUCT, LIST, SET, MAP):
        if t == STRUCT:
            for _ in range(rng.randrange(3) if depth < 4 else 0):
                pos = len(out)
                out += b"\x00\x00\x00"
                ft = w_any(rng, out, depth + 1)
                out[pos] = ft
                out[pos + 1:pos + 3] = struct.pack(">h", rng.randrange(1, 100))
            out.append(0)
        elif t == MAP:
            out += bytes([I32, STRING]) + struct.pack(">i", 1 if depth < 4 else 0)
            if depth < 4:
                w_scalar(rng, I32, out, 0.0)
                w_scalar(rng, STRING, out, 0.0)
        else:
            out += bytes([I32]) + struct.pack(">i", 2)
            w_scalar(rng, I32, out, 0.0)
            w_scalar(rng, I32, out, 0.0)
    else:
        w_scalar(rng, t, out, 0.0)


def w_value(rng, td, out, depth, nan_p=0.0, unknown_p=0.15, keep_p=0.6):
    t = td.type
    if t == STRUCT:
        sd = td.struct
        fields = [f for f in sd.fields if (f.required == T.REQUIRED and rng.random() < 0.97) or rng.random() < keep_p] \
            if depth < 6 else []
        rng.shuffle(fields)
        for f in fields:
            if rng.random() < unknown_p:
                pos = len(out)
                out += b"\x00\x00\x00"
                ut = w_any(rng, out, depth + 1)
                out[pos] = ut
                out[pos + 1:pos + 3] = struct.pack(">h", rng.choice([0, 1000, 2000, -5, 32766]))
            out.append(f.type.type)
            out += struct.pack(">h", f.id)
            w_value(rng, f.type, out, depth + 1, nan_p, unknown_p, keep_p)
        out.append(0)
    elif t in (LIST, SET):
        n = rng.randrange(5) if depth < 6 else 0
        out.append(td.elem.type)
        out += struct.pack(">i", n)
        for _ in range(n):
            w_value(rng, td.elem, out, depth + 1, nan_p, unknown_p, keep_p)
    elif t == MAP:
        n = rng.randrange(4) if depth < 6 else 0
        out += bytes([td.key.type, td.elem.type]) + struct.pack(">i", n)
        for _ in range(n):
            w_value(rng, td.key, out, depth + 1, nan_p, unknown_p, keep_p)
            w_value(rng, td.elem, out, depth + 1, nan_p, unknown_p, keep_p)
    else:
        w_scalar(rng, t, out, nan_p)


def gen_thrift(rng, td, nan_p=0.01, unknown_p=0.1, keep_p=0.6) -> bytes:
    out = bytearray()
    w_value(rng, td, out, 0, nan_p, unknown_p, keep_p)
    return bytes(out)


def mutate(rng, b: bytes) -> bytes:
    """Truncations, corrupted type bytes / sizes, random byte flips."""
    if not b:
        return b
    b = bytearray(b)
    r = rng.random()
    if r < 0.35:
        return bytes(b[:rng.randrange(len(b))])
    if r < 0.55:
        b[rng.randrange(len(b))] = rng.choice([0, 1, 5, 7, 9, 16, 17, 18, 0xFF, 11, 12, 13, 14, 15])
        return bytes(b)
    if r < 0.7 and len(b) >= 4:
        i = rng.randrange(len(b) - 3)
        b[i:i + 4] = struct.pack(">i", rng.choice([-1, -100, 0x7FFFFFFF, 1 << 20]))
        return bytes(b)
    for _ in range(rng.randrange(1, 4)):
        b[rng.randrange(len(b))] = rng.randrange(256)
    return bytes(b)
