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


# ---- the Go-side options: ConvertException, EnableThriftBase, agw.body_dynamic ----
T2J_CONVERT_EXC, T2J_SKIP_RESP_BASE = 1 << 9, 1 << 10


def _example3_svc(opts=None):
    import os
    from schemas import IDL_DIR
    T.init_agw_annos()
    return T.new_descriptor_from_path(os.path.join(IDL_DIR, "example3.thrift"), opts)


def error_resp_thrift():
    """example3.ExampleErrorResp{Int64: 1, Xjson: `{"b":1}`} (FastWrite, id order)."""
    return b"\x0a\x00\x02" + struct.pack(">q", 1) + b"\x0b\x00\x04" + struct.pack(">i", 7) + b'{"b":1}' + b"\x00"


def exception_result_thrift():
    """ExampleServiceExampleMethodResult{Success: ExampleResp{Status: 202},
    Err: Exception{Code: 400, Msg: "this is an exception"}}."""
    succ = (b"\x0b\x00\x01" + struct.pack(">i", 0) + b"\x08\x00\x03" + struct.pack(">i", 202) +
            b"\x0a\x00\x06" + struct.pack(">q", 0) + b"\x04\x7f\xff" + struct.pack(">d", 0.0) + b"\x00")
    msg = b"this is an exception"
    exc = b"\x08\x00\x01" + struct.pack(">i", 400) + b"\x0b\x00\xff" + struct.pack(">i", len(msg)) + msg + b"\x00"
    return b"\x0c\x00\x00" + succ + b"\x0c\x00\x01" + exc + b"\x00"


def test_agw_body_dynamic_read(chk):
    """TestAGWBodyDynamic (conv/t2j/conv_test.go:266-286)."""
    td = _example3_svc().functions()["ErrorMethod"].response().struct.fields[0].type
    fl = T.flatten(td)
    side = T.flatten_t2j(fl)
    assert chk.t2j(fl, side, error_resp_thrift(), T2J_ENABLE_VM) == (0, b'{"Int64":1,"Xjson":{"b":1}}')
    assert chk.t2j(fl, side, error_resp_thrift(), 0) == (0, b'{"Int64":1,"Xjson":"{\\"b\\":1}"}')


def test_convert_exception(chk):
    """TestException (conv/t2j/conv_test.go:310-330): the whole result, the
    error text is the exception's JSON."""
    td = _example3_svc().functions()["ExampleMethod"].response()
    fl = T.flatten(td)
    side = T.flatten_t2j(fl)
    r, js = chk.t2j(fl, side, exception_result_thrift(), T2J_CONVERT_EXC)
    assert r & 0xFF == 11 and js == b'{"code":400,"msg":"this is an exception"}'
    r, js = chk.t2j(fl, side, exception_result_thrift(), 0)  # without the option: both fields as JSON
    assert r == 0 and js.startswith(b'{"":{') and js.endswith(b'"err":{"code":400,"msg":"this is an exception"}}')


def test_response_base_skipped(chk):
    """TestThriftResponseBase (conv/t2j/conv_test.go:232-264): with a context
    BaseResp the root's BaseResp field is skipped and its bytes reported."""
    import json
    import os
    from schemas import IDL_DIR
    td = _example3_svc(T.Options(enable_thrift_base=True)).functions()["ExampleMethod"].response().struct.fields[0].type
    fl = T.flatten(td)
    side = T.flatten_t2j(fl)
    src = open(os.path.join(os.path.dirname(IDL_DIR), "example3resp.bin"), "rb").read()
    r0, js0, _ = chk.t2j2(fl, side, src, 0)
    r1, js1, aux = chk.t2j2(fl, side, src, T2J_SKIP_RESP_BASE)
    assert r0 == 0 and r1 == 0
    a, b = json.loads(js0), json.loads(js1)
    assert "BaseResp" in a and "BaseResp" not in b
    a.pop("BaseResp")
    assert a == b
    lo, hi = aux & 0xFFFFFFFF, aux >> 32
    from dynamicgo_amd.t2j import BaseResp
    br = BaseResp()
    br.fast_read(src[lo:hi])
    want = json.loads(js0)["BaseResp"]
    assert (br.StatusMessage, br.StatusCode) == (want["StatusMessage"], want["StatusCode"])
    assert (br.Extra or {}) == (want.get("Extra") or {})


# ---- more of conv/t2j/conv_test.go's known answers, through the checker ----
T2J_DISALLOW_UNKNOWN = 1 << 4


def api_body_thrift():
    """example3.ExampleApiBody{Code: 1, Code2: 2, InnerCode: {C1: 31, C2: 32,
    C3: [{C1: 41, C2: 42}]}} as FastWriteNocopy writes it (id order; the
    inner element's nil C3 is a default-requiredness list, written empty)."""
    def inner(c1, c2, elems):
        b = b"\x0a\x00\x01" + struct.pack(">q", c1) + b"\x06\x00\x02" + struct.pack(">h", c2)
        return b + b"\x0f\x00\x03\x0c" + struct.pack(">i", len(elems)) + b"".join(elems) + b"\x00"
    return (b"\x0a\x00\x01" + struct.pack(">q", 1) + b"\x06\x00\x02" + struct.pack(">h", 2) +
            b"\x0c\x00\x03" + inner(31, 32, [inner(41, 42, [])]) + b"\x00")


API_BODY_JSON = b'{"Code":1,"code":2,"InnerCode":{"C1":31,"code":32,"C3":[{"C1":41,"code":42,"C3":[]}]}}'


def test_api_body(chk):
    """TestAPIBody (conv/t2j/conv_test.go:288-308): api.body keys are not
    JSON keys on this path; go.tag json names are."""
    td = _example3_svc().functions()["ApiBodyMethod"].response().struct.fields[0].type
    fl = T.flatten(td)
    side = T.flatten_t2j(fl)
    assert chk.t2j(fl, side, api_body_thrift(), T2J_ENABLE_VM) == (0, API_BODY_JSON)


def _example3_resp_bin():
    import os
    from schemas import IDL_DIR
    return open(os.path.join(os.path.dirname(IDL_DIR), "example3resp.bin"), "rb").read()


@pytest.mark.parametrize("which", ["top", "nested"])
def test_unknown_fields(chk, which):
    """TestUnknowFields (conv/t2j/conv_test.go:472-518): example3resp.bin read
    as PartialMethod's response (top) or request (nested) struct: ErrUnknownField
    with DisallowUnknownField, no error without it."""
    fn = _example3_svc().functions()["PartialMethod"]
    td = (fn.response() if which == "top" else fn.request()).struct.fields[0].type
    fl = T.flatten(td)
    side = T.flatten_t2j(fl)
    src = _example3_resp_bin()
    r, _ = chk.t2j(fl, side, src, T2J_DISALLOW_UNKNOWN)
    assert r & 0xFF == 2  # DG_T2J_E_UNKNOWN_FIELD
    r, js = chk.t2j(fl, side, src, 0)
    assert r == 0
    import json
    json.loads(js)


def test_simple_args(chk):
    """TestSimpleArgs (conv/t2j/conv_test.go:711-733): a string and an i64
    response root."""
    fns = _example3_svc().functions()
    for name, src, want in (("String", struct.pack(">i", 5) + b"hello", b'"hello"'),
                            ("I64", struct.pack(">q", 2**63 - 1), b"9223372036854775807")):
        td = fns[name].response().struct.fields[0].type
        fl = T.flatten(td)
        assert chk.t2j(fl, T.flatten_t2j(fl), src, 0) == (0, want)
