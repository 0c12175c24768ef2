"""GPU parity of the flat-struct kernel (j2t_flat.h: field-major, the
default for flat root structs; forced by DG_F_FLAT_PATH) against the
reference's own engine (oracle/_ref), byte for byte and status word for
status word; and against the lane-per-message small kernel
(DG_F_NO_FLAT_PATH) on the same batches."""
import random

import numpy as np
import pytest

import fuzz
import oracle
from dynamicgo_amd import conv, thrift as T, workloads as W
from test_gpu_parity import _raw_batch

pytestmark = pytest.mark.gpu

FLAT = 1 << 19  # DG_F_FLAT_PATH
NO_FLAT = 1 << 21  # DG_F_NO_FLAT_PATH


def _chk():
    return oracle.RefOracle() or oracle.PortOracle()


def flat_desc():
    """A flat struct with every scalar type, binary, js_conv fields,
    required / default / optional fields, an alias and a non-IDL-order id."""
    return T.struct_type("Flat", [
        T.FieldDescriptor(1, "b", T.builtin("bool"), T.OPTIONAL),
        T.FieldDescriptor(2, "y", T.builtin("byte"), T.OPTIONAL),
        T.FieldDescriptor(3, "s16", T.builtin("i16"), T.DEFAULT),
        T.FieldDescriptor(4, "s32", T.builtin("i32"), T.OPTIONAL),
        T.FieldDescriptor(5, "s64", T.builtin("i64"), T.OPTIONAL),
        T.FieldDescriptor(6, "d", T.builtin("double"), T.OPTIONAL),
        T.FieldDescriptor(7, "str", T.builtin("string"), T.OPTIONAL, alias="Str"),
        T.FieldDescriptor(8, "bin", T.builtin("binary"), T.OPTIONAL),
        T.FieldDescriptor(9, "vm64", T.builtin("i64"), T.OPTIONAL, vm=T.VM_JSCONV),
        T.FieldDescriptor(10, "vm16", T.builtin("i16"), T.OPTIONAL, vm=T.VM_JSCONV),
        T.FieldDescriptor(11, "vms", T.builtin("string"), T.OPTIONAL, vm=T.VM_JSCONV),
        T.FieldDescriptor(12, "req", T.builtin("i32"), T.REQUIRED),
        T.FieldDescriptor(40, "far", T.builtin("double"), T.DEFAULT),
    ])


def _compare(flat, msgs, flags):
    chk = _chk()
    bad = []
    outs, rets = _raw_batch(flat, msgs, flags)
    er, eo = chk.j2t_batch(flat, msgs, flags & 0xFFFF)
    for i in range(len(msgs)):
        if int(rets[i]) != int(er[i]) or outs[i] != eo[i]:
            bad.append((i, msgs[i][:120], hex(int(rets[i])), hex(int(er[i]))))
    return bad


@pytest.mark.parametrize("flags", [0x1, 0x0, 0x5, 0x7, 0x41, 0x23, 0x83, 0x11, 0x201])
def test_flat_fuzz_vs_oracle(flags):
    rng = random.Random(500 + flags)
    for td in (flat_desc(), W.simple_desc()):
        fl = T.flatten(td)
        msgs = [fuzz.gen_message(rng, td, mutate_p=rng.random() < 0.3) for _ in range(1500)]
        bad = _compare(fl, msgs, flags | FLAT)
        assert not bad, bad[:4]


def test_flat_clean_messages_stay_on_the_flat_kernel():
    """Well-formed C2 batches: every message is converted by the flat kernel
    (no bail to the list pass), identical to the oracle and to the small
    kernel."""
    ctx = conv.default_context()
    rng = random.Random(42)
    td = W.simple_desc()
    fl = T.flatten(td)
    msgs = W.gen_flat_batch(rng, 20000)
    ctx.stats(reset=True)
    o1, r1 = _raw_batch(fl, msgs, 0x1 | FLAT)
    bails, _ = ctx.stats(reset=True)
    o2, r2 = _raw_batch(fl, msgs, 0x1 | NO_FLAT)
    assert o1 == o2 and list(r1) == list(r2)
    assert not any(int(r) for r in r1)
    assert bails == 0, bails
    assert not _compare(fl, msgs[:3000], 0x1 | FLAT)


@pytest.mark.parametrize("variant", ["c2x", "c2s", "ws", "escapes", "unknown", "dups"])
def test_flat_variants(variant):
    rng = random.Random(7)
    td = W.simple_desc()
    fl = T.flatten(td)
    flags = 0x1
    if variant == "c2x":
        msgs, flags = W.gen_flat_batch(rng, 4000), 0x7
    elif variant == "c2s":
        msgs = W.gen_flat_batch_shuffled(rng, 4000)
    elif variant == "ws":
        msgs = [fuzz.spacify(random.Random(k), m.decode()).encode() for k, m in enumerate(W.gen_flat_batch(rng, 3000))]
        msgs = [b"  \n" + m + b" \t" for m in msgs]
    elif variant == "escapes":
        msgs = [('{"StringField":"a\\nb\\u00e9\\ud83d\\ude00\\t","ByteField":-1,"BinaryField":"%s"}' %
                 rng.choice(["", "QQ==", "QUI=", "QUJD", "QUJDRA==", "QUJDREVG"])).encode() for _ in range(500)]
        msgs += [b'{"StringField":"q\\"x"}', b'{"StringField":"b\\\\"}', b'{"StringField":"\\/"}']
    elif variant == "unknown":
        msgs = [('{"x%d":%s,"I32Field":%d,"zz":"%s","DoubleField":1.5}' %
                 (k, rng.choice(["1", "true", "\"s\"", "[1]", "{}", "null", "-2.5e3"]), k, "v" * (k % 9)))
                .encode() for k in range(2000)]
    else:
        msgs = [('{"I32Field":%d,"I32Field":%d,"StringField":"a","StringField":"bc"}' % (k, -k)).encode()
                for k in range(1000)]
    for extra in (FLAT, 0, NO_FLAT):
        bad = _compare(fl, msgs, flags | extra)
        assert not bad, (extra, bad[:4])


def test_flat_edges():
    td = flat_desc()
    fl = T.flatten(td)
    msgs = [b"", b"{}", b" { } ", b"{", b"}", b'{"req":1}', b'{"req":1,}', b'{,"req":1}', b'{"req":1 "b":true}',
            b'{"req":1}x', b'{"req":1} {}', b'[1]', b'"s"', b'1', b'null', b'{"req":null}', b'{"req":1,"b":nul}',
            b'{"req":1,"Str":"' + b"x" * 400 + b'"}', b'{"req":1,"Str":"' + b"x" * 600 + b'"}',
            b'{"req":1,"str":"by name"}', b'{"req":1,"vm64":"123","vm16":"-7","vms":42}', b'{"req":1,"vm64":""}',
            b'{"req":2147483648}', b'{"req":1,"y":128}', b'{"req":1,"d":1e400}', b'{"req":1,"s64":"5"}',
            b'{"req":1,"bin":"QQ=="}', b'{"req":1,"bin":"QR=="}', b'{"req":1,"bin":"Q==="}', b'{"req":1,"bin":"QQ"}',
            b'{"req":1,"b":true,"b":false}', b'{"\\u0072eq":1}', b'{"req":1,"Str":"\xff\xfe"}',
            b'{"req" : 1 , "far" : 2.5 }', b'{"req":1,"far":-0.0,"s16":32767}',
            b'{"req":1,"bin":"QQ=A"}', b'{"req":1,"bin":"Q=A="}', b'{"req":1,"bin":"QUJDRA=A"}',
            b'{"req":1,"bin":"QUJDREVGR0hJSktMTU5PUFFSU1RVVldYWVo=A"}',
            b'{"req":1,"bin":"QUJDREVGR0hJSktMTU5PUFFSU1RVVldYWVpbXF1eX2BhYmNkZWZnaA=="}',
            b'{"req":1,"Str":"0123456789abcdefghijklmnopqrstuvwxyz0123456789abcdefghij"}']
    for flags in (0x1, 0x0, 0x7, 0x23, 0x5):
        for extra in (FLAT, 0, NO_FLAT):
            bad = _compare(fl, msgs, flags | extra)
            assert not bad, (hex(flags), extra, bad[:4])


def test_flat_lengths_up_to_256():
    """Messages of every length up to the flat kernel's 256-byte limit, at
    every alignment in the arena (structure lanes cover 4 words each; lane 7
    takes word 32 only when a message reaches it), and just past it (listed
    for the wave kernel or the list pass)."""
    td = W.simple_desc()
    fl = T.flatten(td)
    msgs = []
    for n in list(range(180, 262)) + [511, 512, 513]:
        base = '{"ByteField":1,"I32Field":2,"StringField":"%s","I64Field":3}'
        pad = n - len(base % "")
        if pad < 0:
            continue
        m = (base % ("s" * pad)).encode()
        assert len(m) == n
        for lead in range(8):  # leading spaces: every alignment of the braces and words
            msgs.append(b" " * lead + m)
        msgs.append(b'{"StringField":"' + b"," * (n - 19) + b'"}')  # commas inside a string at every word
    for extra in (FLAT, 0, NO_FLAT):
        bad = _compare(fl, msgs, 0x1 | extra)
        assert not bad, (extra, bad[:4])


def _wrap_desc():
    """Mixed-like root: two members of one flat struct type (both wrap),
    one of a non-flat type, a REQUIRED-free rest."""
    inner = W.simple_desc()
    nest = T.struct_type("N", [T.FieldDescriptor(1, "l", T.list_of(T.builtin("i32")), T.OPTIONAL)])
    return T.struct_type("Wrap", [
        T.FieldDescriptor(1, "Flat", inner, T.DEFAULT),
        T.FieldDescriptor(2, "Nested", nest, T.DEFAULT),
        T.FieldDescriptor(4, "Other", inner, T.OPTIONAL, alias="other"),
        T.FieldDescriptor(5, "n", T.builtin("i32"), T.OPTIONAL),
    ])


def _wrap_msgs(rng, k):
    out = []
    for _ in range(k):
        s = W.simple_obj(rng)
        out.append(rng.choice([b'{"Flat":%s}', b'{"other":%s}', b' { "Flat" :\n%s } ', b'{"Other":%s}'])
                   % s.encode())
    return out


def test_flat_wrapped_members_vs_oracle():
    """{"key":{flat}} members of a non-flat root on the flat kernel's wrapped
    mode (FlatParams::wrap): the outer header, the inner fields, two STOPs --
    byte-identical to the reference; every well-formed one stays on the flat
    kernel (no bail); the odd shapes decline to the list pass and still come
    out exact."""
    ctx = conv.default_context()
    rng = random.Random(31)
    td = _wrap_desc()
    fl = T.flatten(td)
    msgs = [m for m in _wrap_msgs(rng, 6000) if len(m) <= 256]
    ctx.stats(reset=True)
    bad = _compare(fl, msgs, 0x1 | FLAT)
    bails, _ = ctx.stats(reset=True)
    assert not bad, bad[:4]
    assert bails == 0, bails
    odd = [b'{"Flat":{}}', b'{"Flat":null}', b'{"Flat":{"ByteField":1},"Flat":{}}', b'{"Fl\\u0061t":{"ByteField":1}}',
           b'{"Nested":{"l":[1,2]}}', b'{"Flat":{"ByteField":1}', b'{"Flat":{"ByteField":1}}}', b'{"zz":{"a":1}}',
           b'{"Flat":{"ByteField":1},"n":3}', b'{"n":3,"Flat":{"ByteField":1}}', b'{"Flat":[1]}', b'{"Flat":{"a":{}}}',
           b'{"Flat":{"ByteField":{}}}', b'{"Flat" {"ByteField":1}}', b'{"Flat":{"ByteField":1} }x',
           b'{"Flat":{"StringField":"}"}}', b'{"Flat":{"StringField":"{"},"x":1}', b'{"Flat":{"I32Field":1,"I32Field":2}}',
           b'{"Flat":{"ByteField":300}}', b'{}', b'{"Flat":{"ByteField":1},}', b'{"Other":{"ByteField":1}}']
    for flags in (0x1, 0x0, 0x3, 0x7, 0x21, 0x81):
        for extra in (FLAT, 0, NO_FLAT):
            bad = _compare(fl, odd + msgs[:300], flags | extra)
            assert not bad, (hex(flags), extra, bad[:4])


def test_flat_wrapped_mixed_batch():
    """A C5-style batch (flat / nested / large members of workloads.Mixed)
    through the default routing: the flat kernel's wrapped mode, the wave
    kernel for the long ones, the list pass -- identical to the reference."""
    rng = random.Random(45)
    td = W.mixed_desc()
    fl = T.flatten(td)
    msgs = W.gen_mixed_batch(rng, 3000, large_scale=0.05)
    assert not _compare(fl, msgs, 0x1)
    assert not _compare(fl, msgs, 0x7)


def test_flat_task_cap_path():
    """More string chunk tasks in one block than FL_MAXTASK (512): the
    messages past the cap decline (their task slots marked empty) and the
    list pass redoes them; the ones within it stay exact (round 3's fault:
    stale task slots past the cap)."""
    td = T.struct_type("Five", [T.FieldDescriptor(k + 1, c, T.builtin("string"), T.OPTIONAL)
                                for k, c in enumerate("abcde")] +
                       [T.FieldDescriptor(6, "z", T.builtin("binary"), T.OPTIONAL)])
    fl = T.flatten(td)
    rng = random.Random(3)
    msgs = []
    for k in range(64 * 20):
        parts = ['"%s":"%s"' % (c, "".join(rng.choice("abcdefgh") for _ in range(33 + (k % 3)))) for c in "abcde"]
        if k % 4 == 0:
            parts.append('"z":"QUJDREVGR0hJSktMTU5PUFFSU1RVVldY"')
        m = ("{" + ",".join(parts) + "}").encode()
        assert len(m) <= 256
        msgs.append(m)
    assert not _compare(fl, msgs, 0x1 | FLAT)


def test_flat_escape_table_vs_oracle():
    """The structure phase's escape table (j2t_flat.h fl_escape): every simple
    escape, \\u of 1, 2 and 3 UTF-8 bytes (upper/lower-case hex), escapes at
    a string's start and end, next to each other, up to FL_NESC (8) per
    message and beyond it (C1's string has 8), in keys, in numbers' js_conv text, in binary
    fields, invalid ones and surrogates (declined to the list pass): the
    bytes and status words of the reference. Escapes the table keeps stay on
    the flat kernel (no bail)."""
    rng = random.Random(77)
    td = W.simple_desc()
    fl = T.flatten(td)
    pieces = ["a", "Z9", "\\n", "\\t", "\\r", "\\b", "\\f", "\\/", "\\u0041", "\\u00e9", "\\u00E9", "\\u07ff",
              "\\u0800", "\\u4e2d", "\\uFFFF", "\\u0000", "é"]
    keep = []
    for _ in range(3000):
        body = "".join(rng.choice(pieces) for _ in range(rng.randint(0, 10)))
        keep.append(('{"ByteField":%d,"StringField":"%s","I32Field":%d}' %
                     (rng.randint(-128, 127), body, rng.randint(-2**31, 2**31 - 1))).encode())
    ok = [m for m in keep if m.count(b"\\") <= 8]
    ctx = conv.default_context()
    ctx.stats(reset=True)
    outs, rets = _raw_batch(fl, ok + [W.c1_simple_json()] * 256, 0x1 | FLAT)
    bails, _ = ctx.stats(reset=True)
    assert bails == 0, bails
    assert not _compare(fl, ok, 0x1 | FLAT)
    odd = [b'{"StringField":"\\ud83d\\ude00"}', b'{"StringField":"\\ud83d"}', b'{"StringField":"\\x"}',
           b'{"StringField":"\\u12"}', b'{"StringField":"\\u12G4"}', b'{"StringField":"ab\\',
           b'{"Str\\u0069ngField":"k"}', b'{"StringField":"\\n\\n\\n\\n\\n"}', b'{"BinaryField":"QQ\\u003d="}',
           b'{"I32Field":1\\n}', b'{"StringField":"\\u002"}', b'{"StringField":"\\n","StringField":"\\t\\b\\f\\r"}',
           b'{"StringField":"' + b"\\u00e9" * 8 + b'"}', b'{"StringField":"' + b"\\u00e9" * 9 + b'"}',
           W.c1_simple_json()]
    for flags in (0x1, 0x11, 0x7):
        for extra in (FLAT, NO_FLAT):
            bad = _compare(fl, keep + odd, flags | extra)
            assert not bad, (hex(flags), extra, bad[:4])


INT_TOKENS = ["0", "-0", "7", "-7", "00", "01", "-01", "-", "--1", "+1", "1-", "12a", "1.", "1.5", "-1.25", "1e5", "1E+2",
              "-0.0", "0e0", "127", "-128", "128", "32767", "-32768", "2147483647", "-2147483648", "2147483648",
              "9223372036854775807", "-9223372036854775808", "9223372036854775808", "-9223372036854775809",
              "9999999999999999999", "18446744073709551615", "18446744073709551616", "12345678901234567890",
              "123456789012345678901", "1234567", "12345678", "123456789", "1234567890123456", "12345678901234567",
              "000000000000000000001", "99999999", "100000000", "4294967296"]


@pytest.mark.parametrize("route", ["flat", "small", "wave"])
def test_integer_tokens_vs_oracle(route):
    """fast_vnumber's fixed-step integer path (j2t_fast.h fast_int_regs,
    register sources: the flat kernel's RSrcL, the wave kernel's RSrc) and
    its fall-backs: every integer shape, the int64 edges, 19- and 20-digit
    values, "-0", leading zeros and non-integers, in every numeric field
    type, against the reference; "wave" pads the message past the wave
    kernel's 512-byte threshold."""
    td = flat_desc()
    fl = T.flatten(td)
    msgs = []
    for v in INT_TOKENS:
        for f in ("y", "s16", "s32", "s64", "d", "vm64", "vm16"):
            pad = ',"Str":"' + "p" * 600 + '"' if route == "wave" else ""
            msgs.append(('{"req":1,"%s":%s%s}' % (f, v, pad)).encode())
            msgs.append(('{"%s":%s,"req":%s%s}' % (f, v, v, pad)).encode())
    extra = {"flat": FLAT, "small": NO_FLAT, "wave": NO_FLAT}[route]
    for flags in (0x1, 0x41, 0x5):
        bad = _compare(fl, msgs, flags | extra)
        assert not bad, (route, hex(flags), bad[:4])


DEC_TOKENS = ["0.0", "-0.0", "0.5", "-0.5", "1.5", "-1.25", "00.5", "01.5", "-01.5", "1.", "-1.", ".5", "-.5", "1.2.3",
              "1..2", "1.5e3", "1.5E-3", "1.5x", "1.x5", "-", "0.000123", "-0.000000000000000001", "0.0000000000000000001",
              "0.00000000000000000001", "123456789.0123456789", "1234567890.123456789", "12345678901234567.89",
              "1234567890123456789.0", "9007199254740993.0", "9007199254740993.5", "-510378.14969714754",
              "722205.81933333166", "-6890.4", "3422.05", "1.7976931348623157", "4.9406564584124654", "2.2250738585072014",
              "0.1", "0.2", "0.3", "123.456", "99999999999999999.9", "1.00000000000000000", "1.000000000000000000",
              "5e-324", "1e309", "-1e309", "1.5.", "12345678901234567890.5"]


@pytest.mark.parametrize("route", ["flat", "small", "wave"])
def test_decimal_tokens_vs_oracle(route):
    """fast_vnumber's fixed-step decimal path (j2t_fast.h fast_dec_regs:
    -?D+.D+ with at most 19 digits, mantissa and exponent without the digit
    loops) and its fall-backs to the general path: leading zeros, a point at
    either end, two points, exponents, 19/20/21 digits, the doubles next to
    2^53 and the range edges, in every numeric field type, against the
    reference; "wave" pads the message past the wave kernel's threshold."""
    td = flat_desc()
    fl = T.flatten(td)
    msgs = []
    for v in DEC_TOKENS:
        for f in ("y", "s16", "s32", "s64", "d", "vm64", "vm16", "far"):
            pad = ',"Str":"' + "p" * 600 + '"' if route == "wave" else ""
            msgs.append(('{"req":1,"%s":%s%s}' % (f, v, pad)).encode())
            msgs.append(('{"%s":%s,"req":2%s}' % (f, v, pad)).encode())
    extra = {"flat": FLAT, "small": NO_FLAT, "wave": NO_FLAT}[route]
    for flags in (0x1, 0x41, 0x5):
        bad = _compare(fl, msgs, flags | extra)
        assert not bad, (route, hex(flags), bad[:4])


def test_decimal_map_keys_and_values_vs_oracle(knob):
    """Decimal tokens as numeric map keys (parsed as a prefix: trailing text
    after the number is ignored) and as map/list values, on the wave kernel
    (wave_min 0) and the lane kernel, against the reference."""
    td = T.struct_type("M", [
        T.FieldDescriptor(1, "md", T.map_of(T.builtin("i64"), T.builtin("double")), T.OPTIONAL),
        T.FieldDescriptor(2, "ld", T.list_of(T.builtin("double")), T.OPTIONAL),
        T.FieldDescriptor(3, "mi", T.map_of(T.builtin("double"), T.builtin("i32")), T.OPTIONAL),
    ])
    fl = T.flatten(td)
    msgs = []
    for v in DEC_TOKENS:
        msgs.append(('{"md":{"%s":%s,"7":1.25},"ld":[%s,0.5]}' % (v, v, v)).encode())
        msgs.append(('{"mi":{"%s":1,"%s7":2},"ld":[1.5,%s]}' % (v, v, v)).encode())
    for wm in (0, 512):
        knob("wave_min", wm)
        for flags in (0x1, 0x41):
            bad = _compare(fl, msgs, flags)
            assert not bad, (wm, hex(flags), bad[:4])


def test_flat_field_remap_shuffled_keys():
    """Shuffled key order (c2s): the key pass maps each position to its
    field and every wave converts one FIELD of its 64 messages
    (j2t_flat.h 2a). No message leaves the flat kernel, and the bytes are
    the small kernel's and the reference's; blocks with a duplicate key, an
    unknown key or a malformed field fall back to positions."""
    ctx = conv.default_context()
    rng = random.Random(9)
    td = W.simple_desc()
    fl = T.flatten(td)
    msgs = W.gen_flat_batch_shuffled(rng, 12000)
    ctx.stats(reset=True)
    o1, r1 = _raw_batch(fl, msgs, 0x1 | FLAT)
    bails, _ = ctx.stats(reset=True)
    o2, r2 = _raw_batch(fl, msgs, 0x1 | NO_FLAT)
    assert o1 == o2 and list(r1) == list(r2)
    assert bails == 0, bails
    assert not _compare(fl, msgs[:3000], 0x1 | FLAT)
    mixed = list(msgs[:640])
    for i in range(0, 640, 67):
        mixed[i] = mixed[i].replace(b'"I32Field"', b'"ByteField"', 1)  # a duplicate key
    for i in range(5, 640, 131):
        mixed[i] = mixed[i].replace(b'"I64Field"', b'"Nope"', 1)  # an unknown key
    for i in range(9, 640, 97):
        mixed[i] = mixed[i].replace(b'":', b'" :', 1)
    for flags in (0x1, 0x11, 0x7):
        bad = _compare(fl, mixed, flags | FLAT)
        assert not bad, (hex(flags), bad[:4])
