"""GPU: the wave-per-message token-parallel kernel (j2t_wave.h).

Every case is checked byte-for-byte (Thrift bytes + packed status word)
against the oracle; the cases in MUST_WAVE must also stay on the wave path
(no bail to the exact machine), so that the grammar the kernel claims to
handle is really handled by it — including tokens and strings that straddle
the 64-token pages and the 256-byte scan chunks."""
import json
import random

import pytest

import fuzz
import oracle
from dynamicgo_amd import conv, thrift as T, workloads as W

from test_gpu_parity import _raw_batch, NO_WAVE

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["4", "5"], ids=["occ4", "occ5"])
def all_messages_on_the_wave_kernel(knob, request):
    """Route every message (not only those > 512 B) to the wave kernel, once
    through each of its two instances (4 and 5 waves/SIMD, j2t_wave.h)."""
    knob("wave_min", 0)
    knob("wave_occ", request.param)


def _checker():
    return oracle.RefOracle() or oracle.PortOracle()


def _simple(**kw):
    d = {"ByteField": 1, "I64Field": 2, "DoubleField": 1.5, "I32Field": 3, "StringField": "s", "BinaryField": "aGk="}
    d.update(kw)
    return d


def _must_wave_cases():
    rng = random.Random(11)
    cases = []
    cases.append(json.dumps(_simple()).encode())
    cases.append(json.dumps(_simple(), indent=4).encode())                     # whitespace everywhere
    cases.append(b'{"ByteField":1,"StringField":"' + b"x" * 700 + b'"}')       # string over 2 scan chunks
    cases.append(b'{"StringField":"' + b"a\\\\" * 40 + b'\\"q"}')              # backslash runs at every lane phase
    cases.append(b'{"StringField":"' + b"\\\\\\\\" * 30 + b'","ByteField":5}')  # runs of 4 backslashes
    for k in range(8):                                                        # escape across each lane offset
        cases.append(b'{"StringField":"' + b"y" * k + b'\\"\\n\\u00e9\\ud83d\\ude00z","I32Field":-7}')
    cases.append(b'{"ByteField":null,"I64Field":null,"StringField":null}')      # null struct fields
    cases.append(b'{"Zzz":{"a":[1,2,{"b":null}],"c":"d"},"ByteField":3,"Q":[[],[[]],{}]}')  # skipped values
    cases.append(b'{"BinaryField":"' + b"QUJD" * 300 + b'"}')                  # long base64
    cases.append(b'{"BinaryField":"QQ=="}')
    cases.append(b'{"BinaryField":"QUI="}')
    cases.append(b'{"BinaryField":""}')
    for n in (28, 32, 36, 60, 64, 68, 92, 96, 100):                           # base64 chunk-task boundaries
        cases.append(b'{"ByteField":2,"BinaryField":"' + (b"QUJD" * 40)[:n - 4] + b'QQ==","I32Field":1}')
    for n in (7, 8, 9, 31, 32, 33, 63, 64, 65, 100):                          # copy chunk-task boundaries
        cases.append(b'{"StringField":"' + bytes(97 + (i % 26) for i in range(n)) + b'","ByteField":4}')
    for k in range(240, 262):                                                 # escapes counted by the scan:
        cases.append(b'{"StringField":"' + b"z" * k + b'\\n\\t\\"\\\\\\/\\b\\f\\r end","I32Field":3}')  # letter in the next chunk
    cases.append(b'{"StringField":"' + b"\\n" * 300 + b'","ByteField":1}')   # 300 escapes in one string
    cases.append(b'{"StringField":"\\u0041\\n","BinaryField":"QUI="}')          # \u with a simple one
    # long-string mode (bodies past WV_LONG = 1024 bytes are written while the
    # scan reads them): lengths around the threshold and every 4-byte phase
    # of the quote, base64 with and without padding, plain strings, two long
    # strings in one message, a long value after many entries
    for n in (1016, 1020, 1024, 1028, 1280, 4096, 20000):
        for ph in range(4):
            cases.append(b'{' + b' ' * ph + b'"BinaryField":"' + (b"QUJD" * (n // 4))[:n - 4] + b'QQ==",'
                         b'"StringField":"' + bytes(97 + (i * 7 + ph) % 26 for i in range(n + ph)) + b'","ByteField":3}')
    cases.append(b'{"BinaryField":"' + b"QUJD" * 700 + b'"}')                     # no padding
    cases.append(b'{"BinaryField":"' + b"QUJD" * 700 + b'QUI="}')
    cases.append(b'{"ByteField":1' + b"".join(b',"K%d":%d' % (i, i) for i in range(100)) + b',"StringField":"' +
                 b"w" * 3000 + b'"}')
    cases.append(b'{"StringField":"' + b"s" * 1500 + b'","StringField2":"' + b"t" * 1500 + b'"}')  # unknown key: skipped
    cases.append(("nest", b'{"ListString":["' + b"l" * 3000 + b'"],"String":"' + b"m" * 2000 + b'",'
                  b'"MapStringString":{"k":"' + b"v" * 2500 + b'"},"SimpleStruct":{"BinaryField":"'
                  + b"QUJD" * 600 + b'","StringField":"' + b"q" * 1200 + b'"},"Binary":"' + b"QUJD" * 400 + b'"}'))
    cases.append(b'{"DoubleField":-0,"I64Field":-9223372036854775808,"I32Field":1.9,"ByteField":-129}')
    cases.append(b'{"DoubleField":1e22,"I64Field":123456789012345678,"I32Field":2147483648}')
    cases.append(b'{"DoubleField":0.1e-5,"I64Field":99999999999999999999}')   # overflow -> double -> cvt
    for num in (b"2.2250738585072011e-308", b"4.9406564584124654e-324", b"9007199254740993",
                b"1.00000000000000011102230246251565404236316680908203125", b"7.2057594037927933e+16",
                b"123456789012345678901234567890e-10", b"0.1000000000000000055511151231257827021181583404541015625",
                b"-1797693134862315708145274237317043567980705675258449965989174768031572607800285387605895586"
                b"3276687817154045895351438246423432132688946418276846754670353751698604991057655128207624549009"
                b"03893289261371104e-00"):
        cases.append(b'{"DoubleField":' + num + b',"I64Field":' + num + b'}')   # slow-path (big decimal) numbers
    nest = {"String": "s", "ListSimple": [_simple() for _ in range(30)], "Double": 2.25, "I32": 7,
            "ListI32": list(range(150)), "I64": -1, "MapStringString": {"k%d" % i: "v%d" % i for i in range(40)},
            "SimpleStruct": _simple(StringField=None), "MapI32I64": {str(i): i * 3 for i in range(-5, 50)},
            "ListString": ["a" * i for i in range(70)], "Binary": "AAEC", "MapI64String": {"-5": "x", "12": None},
            "ListI64": [1, None, 3], "Byte": 9, "MapStringSimple": {"a": _simple(), "b": None, "c": {}}}
    cases.append(("nest", json.dumps(nest).encode()))
    cases.append(("nest", json.dumps(nest, indent=2).encode()))
    cases.append(("nest", b'{"ListI32":[],"MapI32I64":{},"ListSimple":[{},{}],"MapStringSimple":{"":{}}}'))
    cases.append(("nest", b'{"MapI32I64":{"12abc":1,"-3":2}}'))                # numeric key: trailing text ignored
    for _ in range(20):
        cases.append(("nest", W.nesting_obj(rng).encode()))
    return cases


def _may_bail_cases():
    return [
        b'{"ByteField":1,"ByteField":2}',            # duplicate key
        b'{"Byte\\u0046ield":1}',                    # escaped key
        b'{"ByteField":1} trailing "junk',
        b'{"ByteField":01}', b'{"ByteField":1,}', b'{"ByteField" 1}', b'{"ByteField":tru}', b'{"ByteField":[1]}',
        b'{"StringField":"abc', b'{"BinaryField":"QQ"}', b'{"BinaryField":"Q\\nQ=="}', b'{"DoubleField":1e400}',
        b'{"BinaryField":"QQ=A"}', b'{"BinaryField":"' + b"QUJD" * 20 + b'QQ=A"}',   # '=' then a letter: decode error
        b'{"StringField":"\\ud800"}', b'{"StringField":"\\x"}', b"[1]", b"", b"null", b"  {}  ", b"{",
        b'{"ByteField":1]', b'{"a":[1,2}', b'{"ByteField":1e2}', b'{"I32Field":"12"}',
        b'{"ByteField":1,,"I32Field":2}', b'{"ByteField"::1}', b'{"ByteField":1,:"I32Field":2}',  # two separators
        b'{"ByteField":1' + b":" * 256 + b'"I32Field":2}',                  # 256 colons (not one comma)
        b'{"StringField":"a\\n"' + b"," * 256 + b'}',                       # 256 commas after an escaped string
        b'{"StringField":"a\\n"' + b"," * 255 + b'"I32Field":2}',
        b'{"StringField":"\\q\\n"}', b'{"StringField":"\\n\\u12"}',
        # long-string mode: errors and escapes after the stream started
        b'{"BinaryField":"' + b"QUJD" * 500 + b'Q!JD' + b"QUJD" * 100 + b'"}',   # a bad character
        b'{"BinaryField":"' + b"QUJD" * 500 + b'QQ==' + b"QUJD" * 100 + b'"}',   # padding in the middle
        b'{"BinaryField":"' + b"QUJD" * 500 + b'QQ=A"}', b'{"BinaryField":"' + b"QUJD" * 500 + b'QUJ"}',
        b'{"BinaryField":"' + b"QUJD" * 500 + b'\\n"}',
        b'{"StringField":"' + b"e" * 1800 + b'\\n\\t' + b"f" * 900 + b'","ByteField":2}',  # escapes: page writes it
        b'{"StringField":"' + b"e" * 1800 + b'\\u00e9' + b"f" * 900 + b'"}',
        b'{"StringField":"' + b"x" * 3000,                                     # unterminated
        b'{"ByteField":1,"ByteField":2,"StringField":"' + b"d" * 2000 + b'"}',  # duplicate before it
        b'{"StringField":"' + b"d" * 2000 + b'","StringField":"z"}',           # duplicate after it
    ]


def _run(fl, msgs, flags=1):
    ctx = conv.default_context()
    ctx.stats(reset=True)
    outs, rets = _raw_batch(fl, msgs, flags)
    bails, _ = ctx.stats(reset=True)
    return outs, rets, bails


def test_wave_path_handles_valid_grammar():
    simple = T.flatten(W.simple_desc())
    nest = T.flatten(W.nesting_desc())
    chk = _checker()
    groups = {"simple": [], "nest": []}
    for c in _must_wave_cases():
        if isinstance(c, tuple):
            groups[c[0]].append(c[1])
        else:
            groups["simple"].append(c)
    for name, fl in (("simple", simple), ("nest", nest)):
        msgs = groups[name]
        outs, rets, bails = _run(fl, msgs)
        for m, o, r in zip(msgs, outs, rets):
            assert (int(r), o) == chk.j2t(fl, m, 1), m[:200]
        assert bails == 0, name


def test_wave_path_bails_are_exact():
    fl = T.flatten(W.simple_desc())
    chk = _checker()
    msgs = _may_bail_cases()
    for flags in (1, 0, 0x23, 0x11):
        outs, rets, _ = _run(fl, msgs, flags)
        for m, o, r in zip(msgs, outs, rets):
            assert (int(r), o) == chk.j2t(fl, m, flags), (hex(flags), m)


def test_wave_vs_lane_kernel_on_mixed_batch():
    """C5-style mixed batch (flat + nested + large) through both kernels,
    and against the reference (not a self-comparison only)."""
    fl = T.flatten(W.mixed_desc())
    msgs = W.gen_mixed_batch(random.Random(45), 3000, large_scale=0.1)
    o1, r1, b1 = _run(fl, msgs, 1)
    o2, r2, _ = _run(fl, msgs, 1 | NO_WAVE)
    assert list(r1) == list(r2)
    assert o1 == o2
    assert b1 == 0
    er, eo = _checker().j2t_batch(fl, msgs, 1)
    assert [int(r) for r in r1] == [int(r) for r in er]
    assert list(o1) == list(eo)


@pytest.mark.parametrize("flags", [0x3, 0x7])
def test_default_writes_on_nested_descriptors_vs_oracle(flags):
    """WRITE_DEFAULT (0x2) on nested structs: unset fields, containers and
    nested defaults are written, so "{}" grows to 120 bytes -- past the batch
    checker's slot, which hid these cases until tools/fuzz_sweep.py (the
    checker now redoes them alone). Every route vs the reference."""
    chk = _checker()
    for td in (W.nesting_i64_desc(), W.mixed_desc()):
        fl = T.flatten(td)
        rng = random.Random(31 + flags)
        msgs = [b"{}", b'{"I32":5}', b'{"Nested":{}}', b'{"Flat":{},"Nested":{}}'] + \
               [fuzz.gen_message(rng, td, mutate_p=rng.random() < 0.2) for _ in range(600)]
        er, eo = chk.j2t_batch(fl, msgs, flags)
        for extra in (0, NO_WAVE):
            outs, rets = _raw_batch(fl, msgs, flags | extra)
            bad = [i for i in range(len(msgs)) if int(rets[i]) != int(er[i]) or outs[i] != eo[i]]
            assert not bad, (hex(flags), extra, msgs[bad[0]][:120])
