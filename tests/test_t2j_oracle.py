"""CPU: the t2j checker (the C restatement of conv/t2j over the reference's
own native quote/i64toa/f64toa/b64encode, oracle/ref_harness.c) against the
reference's own known answers (conv/t2j/conv_test.go:332-386,
TestInt2String)."""
import math
import struct

import pytest

import oracle
from dynamicgo_amd import thrift as T
from schemas import idl_desc

T2J_BYTE_AS_UINT8, T2J_INT64_AS_STRING, T2J_NULL_FOR_NAN_INF = 1, 2, 4
T2J_ENABLE_VM = 1 << 8


def int2float_thrift(subfix=0.92653):
    """example3.ExampleInt2Float{Int32: 1, Float64: 3.14, String_: "hello",
    Int64: 2, Subfix: subfix}, fields in id order (kitex FastWrite)."""
    b = b"\x08\x00\x01" + struct.pack(">i", 1)
    b += b"\x04\x00\x02" + struct.pack(">d", 3.14)
    b += b"\x0b\x00\x03" + struct.pack(">i", 5) + b"hello"
    b += b"\x0a\x00\x04" + struct.pack(">q", 2)
    b += b"\x04\x7f\xff" + struct.pack(">d", subfix)
    return b + b"\x00"


@pytest.fixture(scope="module")
def chk():
    o = oracle.RefT2JOracle()
    if o is None:
        pytest.skip("oracle/_ref not built")
    return o


def test_int2string_known_answers(chk):
    td = idl_desc("example3.thrift", "Int2FloatMethod")
    fl = T.flatten(td)
    side = T.flatten_t2j(fl)
    src = int2float_thrift()
    assert chk.t2j(fl, side, src, T2J_ENABLE_VM) == (
        0, '{"Int32":"1","Float64":"3.14","中文":"hello","Int64":2,"Subfix":0.92653}'.encode())
    assert chk.t2j(fl, side, src, 0) == (
        0, '{"Int32":1,"Float64":3.14,"中文":"hello","Int64":2,"Subfix":0.92653}'.encode())
    assert chk.t2j(fl, side, src, T2J_INT64_AS_STRING) == (
        0, '{"Int32":1,"Float64":3.14,"中文":"hello","Int64":"2","Subfix":0.92653}'.encode())
    nan = int2float_thrift(math.nan)
    r, _ = chk.t2j(fl, side, nan, 0)
    assert r & 0xFF == 5  # ErrWrite: encounter Nan or Inf double
    assert chk.t2j(fl, side, nan, T2J_NULL_FOR_NAN_INF) == (
        0, '{"Int32":1,"Float64":3.14,"中文":"hello","Int64":2,"Subfix":null}'.encode())


def test_roundtrip_of_j2t_goldens(golden, chk):
    """Every successful golden j2t output converts back; t2j(j2t(x)) is
    valid JSON whose keys are the fields' aliases."""
    import json
    rows, flats = golden
    n = 0
    for name, flags, js, ret, out in rows:
        if ret != 0 or name in ("string_root", "i64_root") or not out:
            continue
        fl = flats[name]
        # the golden fixture holds the blob only; the side table needs the
        # field objects, so rebuild from the schema for the IDL descriptors
        if not hasattr(fl, "fields"):
            continue
        r, j = chk.t2j(fl, T.flatten_t2j(fl), out, 0)
        assert r == 0
        json.loads(j)
        n += 1


def test_generated_messages(chk):
    """The t2j test generator (tests/t2jgen.py) drives every branch of the
    checker: successful messages parse as JSON with the fields' aliases as
    keys; mutated ones produce the read / type / NaN error codes."""
    import json
    import random
    import t2jgen
    td = t2jgen.all_types_desc()
    fl = T.flatten(td)
    side = T.flatten_t2j(fl)
    rng = random.Random(7)
    codes = {}
    ok = 0
    for i in range(400):
        m = t2jgen.gen_thrift(rng, td)
        if i % 2:
            m = t2jgen.mutate(rng, m)
        r, j = chk.t2j(fl, side, m, 0)
        codes[r & 0xFF] = codes.get(r & 0xFF, 0) + 1
        if r == 0:
            json.loads(j.decode("utf-8", "replace"))
            ok += 1
    assert ok > 150
    assert {1, 3}.issubset(codes), codes  # ErrRead, ErrDismatchType
