"""t2j EnableHttpMapping, host side (CPU): dynamicgo_amd.t2j's writeHttpValue
serving loop run over the C harness (oracle/ref_harness.c dgref_t2j3, the
same stop/answer protocol as the device) instead of the GPU, against the
reference's own t2j HTTP-mapping tests (conv/t2j/conv_test.go:388-771,
conv/t2j/conv_amd64_test.go:32-85). tests/test_gpu_t2j.py runs the same
cases on the device and compares each stop with the harness."""
import json
import math
import random
import struct

import numpy as np
import pytest

import oracle
from dynamicgo_amd import conv, http as H, t2j, thrift as T
from test_t2j_oracle import _example3_svc


@pytest.fixture(scope="module")
def chk():
    o = oracle.RefT2JOracle()
    if o is None:
        pytest.skip("oracle/_ref not built")
    return o


def harness_conv(chk, opts: conv.Options) -> t2j.BinaryConv:
    """A BinaryConv whose device batch is the C harness (test-only)."""
    cv = t2j.BinaryConv(opts)

    def _batch(desc, msgs, with_base=False, answers=None):
        flat = cv._flat(desc)
        side = T.flatten_t2j(flat)
        o = t2j.to_t2j_opts(cv.opts, with_base)
        outs, rets, auxs = [], [], []
        for k, m in enumerate(msgs):
            r, js, aux = chk.t2j3(flat, side, bytes(m), o, bytes(answers[k]) if answers is not None else b"")
            outs.append(js)
            rets.append(r)
            auxs.append(aux)
        return outs, np.array(rets, dtype=np.uint64), (np.array(auxs, dtype=np.uint64) if with_base else None)

    cv._batch = _batch
    return cv


# ---- Thrift binary writers for the fixtures (kitex FastWrite order) ----
def fld(t: int, fid: int, payload: bytes) -> bytes:
    return bytes([t]) + struct.pack(">h", fid) + payload


def tstr(b) -> bytes:
    b = b.encode() if isinstance(b, str) else b
    return struct.pack(">i", len(b)) + b


def json_object(a: str, b: int) -> bytes:
    """example3.JSONObject{A, B} (k-example3.go:1517-1540)."""
    return fld(11, 1, tstr(a)) + fld(3, 2, struct.pack(">b", b)) + b"\x00"


def resp_desc(method: str, opts=None):
    """thrift.FnResponse (thrift/test_util.go:41-44): field 0's type."""
    return _example3_svc(opts).functions()[method].response().struct.fields[0].type


def test_http_mapping_fallback(chk):
    """TestHttpMappingFallback (conv/t2j/conv_test.go:388-436)."""
    desc = resp_desc("FallbackMethod")
    data = fld(11, 2, tstr("hello")) + fld(11, 3, tstr("world")) + b"\x00"
    for fallback, exp in ((False, b"{}"), (True, b'{"Msg":"hello"}')):
        cv = harness_conv(chk, conv.Options(EnableHttpMapping=True, WriteHttpValueFallback=fallback,
                                            OmitHttpMappingErrors=True))
        resp = H.HTTPResponse()
        assert cv.do(desc, data, resp) == exp
        assert resp.headers["Heeader"][0] == "world"


def test_write_empty(chk):
    """TestWriteEmpty (conv/t2j/conv_test.go:438-470): Status 23 goes to the
    status code, the JSON holds Status 0 (handleUnsets' default) and an empty
    BaseResp."""
    desc = resp_desc("ExampleMethod")
    data = fld(8, 3, struct.pack(">i", 23)) + b"\x00"
    cv = harness_conv(chk, conv.Options(WriteDefaultField=True, EnableHttpMapping=True))
    resp = H.HTTPResponse()
    out = json.loads(cv.do(desc, data, resp))
    assert out.get("Status", 0) == 0
    assert resp.status_code == 23
    # json.Unmarshal into *base.BaseResp: absent members stay zero
    assert {"StatusMessage": "", "StatusCode": 0, **out["BaseResp"]} == {"StatusMessage": "", "StatusCode": 0}


@pytest.mark.parametrize("nob64", [False, True])
def test_nobody_required_fields(chk, nob64):
    """TestNobodyRequiredFields (conv/t2j/conv_test.go:520-568): the binary
    header base64-encoded unless NoBase64Binary."""
    import base64
    desc = resp_desc("Base64BinaryMethod")
    data = fld(11, 1, tstr(b"hello")) + fld(11, 2, tstr(b"world")) + b"\x00"
    cv = harness_conv(chk, conv.Options(EnableHttpMapping=True, NoBase64Binary=nob64))
    resp = H.HTTPResponse()
    out = json.loads(cv.do(desc, data, resp))
    if nob64:
        assert out["Binary"] == "hello"
        assert resp.headers["Binary2"][0] == "world"
    else:
        assert base64.b64decode(out["Binary"]) == b"hello"
        assert resp.headers["Binary2"][0] == base64.b64encode(b"world").decode()


def json_string_data() -> bytes:
    """example3.ExampleJSONString as TestJSONString builds it (FastWrite,
    k-example3.go:1627-1690: Query nil -> an empty struct)."""
    return (fld(12, 1, b"\x00") + fld(15, 2, b"\x0b" + struct.pack(">i", 0)) +
            fld(12, 3, json_object("1", -1)) +
            fld(13, 4, b"\x08\x0b" + struct.pack(">i", 1) + struct.pack(">i", 1) + tstr("1")) +
            fld(12, 5, json_object("", 0)) +
            fld(14, 6, b"\x08" + struct.pack(">i", 2) + struct.pack(">ii", 1, 2)) + b"\x00")


def test_json_string(chk):
    """TestJSONString (conv/t2j/conv_test.go:570-605): container values go
    to headers and cookies as JSON; the query-mapped ones (not supported for
    responses, the errors omitted) fall back into the body."""
    desc = resp_desc("JSONStringMethod")
    cv = harness_conv(chk, conv.Options(EnableHttpMapping=True, WriteHttpValueFallback=True,
                                        OmitHttpMappingErrors=True))
    resp = H.HTTPResponse()
    assert cv.do(desc, json_string_data(), resp) == b'{"Query":{},"Query2":[]}'
    assert json.loads(resp.get_header("header")) == {"a": "1", "b": -1}
    assert {int(k): v for k, v in json.loads(resp.get_header("header2")).items()} == {1: "1"}
    assert json.loads(resp.cookies()[1][1]) == [1, 2]
    assert resp.cookies()[0] == ("cookie", '{a:,b:0}')  # '"' dropped, quoted for the ','


def test_kitex_api_header(chk):
    """TestConvThrift2HTTP_KitexApiHeader (conv/t2j/conv_test.go:735-771):
    UseKitexHttpEncoding prints the values the way kitex does."""
    desc = resp_desc("JSONStringMethod")
    cv = harness_conv(chk, conv.Options(EnableHttpMapping=True, WriteHttpValueFallback=True,
                                        OmitHttpMappingErrors=True, UseKitexHttpEncoding=True))
    resp = H.HTTPResponse()
    assert cv.do(desc, json_string_data(), resp) == b'{"Query":{},"Query2":[]}'
    assert resp.get_header("header") == "map[a:1 b:-1]"
    assert resp.get_header("header2") == "map[1:1]"
    assert resp.cookies()[0][1] == "map[a: b:0]"
    assert resp.cookies()[1][1] == "1,2"


@pytest.mark.parametrize("use_default", [True, False])
def test_default_value(chk, use_default):
    """TestDefaultValue (conv/t2j/conv_test.go:607-653): handleUnsets sends
    the unset mapped fields' defaults to the response."""
    desc = resp_desc("DefaultValueMethod", T.Options(use_default_value=use_default))
    cv = harness_conv(chk, conv.Options(EnableHttpMapping=True, WriteDefaultField=True))
    resp = H.HTTPResponse()
    out = json.loads(cv.do(desc, b"\x00", resp))
    if use_default:
        assert out == {"A": "hello", "B": 1}
        assert resp.get_header("c") == "1.2"
        assert resp.cookies()[0][1] == "const string"
    else:
        assert out == {"A": "", "B": 0}
        assert resp.get_header("c") == "0"
        assert resp.cookies()[0][1] == ""


def test_optional_default_value(chk):
    """TestOptionalDefaultValue (conv/t2j/conv_test.go:655-709)."""
    desc = resp_desc("OptionalDefaultValueMethod", T.Options(use_default_value=True))
    cv = harness_conv(chk, conv.Options(EnableHttpMapping=True, WriteRequireField=True))
    resp = H.HTTPResponse()
    out = json.loads(cv.do(desc, b"\x00", resp))
    assert out == {"B": 1}  # optional A and C stay unset (exp.A = "", exp.C = 0)
    assert resp.cookies()[0][1] == "const string"
    desc = resp_desc("OptionalDefaultValueMethod", T.Options(use_default_value=True, set_optional_bitmap=True))
    cv = harness_conv(chk, conv.Options(EnableHttpMapping=True, WriteRequireField=True, WriteDefaultField=True,
                                        WriteOptionalField=True))
    resp = H.HTTPResponse()
    out = json.loads(cv.do(desc, b"\x00", resp))
    assert out == {"A": "hello", "B": 1, "E": ""}
    assert resp.get_header("c") == "1.2"
    assert resp.cookies()[0][1] == "const string"
    assert resp.get_header("f") == ""


def a_in_b(a, b) -> bool:
    """checkAInB (conv/t2j/conv_test.go:177-240), JSConv relaxed."""
    if not a:
        return True
    if isinstance(a, dict):
        return isinstance(b, dict) and all(k in b and a_in_b(v, b[k]) for k, v in a.items())
    if isinstance(a, list):
        return isinstance(b, list) and len(a) <= len(b) and all(a_in_b(x, y) for x, y in zip(a, b))
    if a == b:
        return True
    try:
        return float(a) == float(b)
    except (TypeError, ValueError):
        return False


def test_conv_thrift2http(chk):
    """TestConvThrift2HTTP (conv/t2j/conv_amd64_test.go:32-85): the reference
    fixture example3resp.bin; two headers (Heeader, Set-Cookie), the root's
    cookie and the InnerBase's String cookie; done twice on fresh
    responses."""
    import os
    g = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    desc = resp_desc("ExampleMethod")
    data = open(os.path.join(g, "example3resp.bin"), "rb").read()
    exp = json.load(open(os.path.join(g, "example3resp.json")))
    cv = harness_conv(chk, conv.Options(EnableValueMapping=True, EnableHttpMapping=True,
                                        OmitHttpMappingErrors=True))
    for _ in range(2):
        resp = H.HTTPResponse()
        out = json.loads(cv.do(desc, data, resp))
        assert a_in_b(out, exp)
        assert resp.headers["Heeader"][0] == "true"
        assert len(resp.headers) == 2, resp.headers
        ck = resp.cookies()
        assert ck[0][0] == "cookie"
        assert ck[1] == ("inner_string", "hello")


def test_errors(chk):
    """Errors: no response object (ErrInvalidParam, conv/t2j/conv.go:62-64);
    a Response error not omitted (errNotImplemented -> ErrUnsupportedType);
    a bad http_code (strconv.Atoi) wrapped as ErrConvert."""
    desc = resp_desc("FallbackMethod")
    data = fld(11, 2, tstr("hello")) + fld(11, 3, tstr("world")) + b"\x00"
    cv = harness_conv(chk, conv.Options(EnableHttpMapping=True))
    with pytest.raises(H.ConvError) as ei:
        cv.do(desc, data, None)
    assert ei.value.behavior == "ErrInvalidParam"
    with pytest.raises(H.ConvError) as ei:
        cv.do(desc, data, H.HTTPResponse())
    assert ei.value.behavior == "ErrUnsupportedType"
    ex = resp_desc("ExampleMethod")
    bad = fld(8, 3, struct.pack(">i", 7)) + b"\x00"
    resp = H.HTTPResponse()
    assert json.loads(harness_conv(chk, conv.Options(EnableHttpMapping=True)).do(ex, bad, resp)) is not None
    assert resp.status_code == 7


def test_f64toa_matches_native(chk):
    """t2j.f64toa (the text of a DOUBLE header) against the reference's native
    f64toa through the harness, over every format branch."""
    td = T.struct_type("D", [(1, "d", T.builtin("double"))])
    fl = T.flatten(td)
    side = T.flatten_t2j(fl)
    rng = random.Random(5)
    vals = [0.0, -0.0, 1.0, -1.5, 0.1, 1e-7, 1.5e-7, 123456.789, 1e20, 1e21, 1.2345e21, 2.0 ** 53, 2.0 ** 60,
            5e-324, 1.7976931348623157e308, 1e-6, 9.999e-7, 100.0, 3.14]
    vals += [rng.uniform(-1e6, 1e6) for _ in range(300)]
    vals += [math.ldexp(rng.random(), rng.randint(-1074, 1023)) for _ in range(300)]
    for v in vals:
        r, js = chk.t2j(fl, side, b"\x04\x00\x01" + struct.pack(">d", v) + b"\x00", 0)
        assert r == 0
        assert js == b'{"d":' + t2j.f64toa(v).encode() + b"}", v


def test_go_formats():
    """fmt %v / strconv 'f' float text the kitex string uses."""
    assert t2j._go_g(1000000.0) == "1e+06"
    assert t2j._go_g(123456.0) == "123456"
    assert t2j._go_g(0.0001) == "0.0001"
    assert t2j._go_g(0.00001) == "1e-05"
    assert t2j._go_g(-1.5) == "-1.5"
    assert t2j._go_f(1e21) == "1000000000000000000000"
    assert t2j._go_f(1e-7) == "0.0000001"
    assert H.cookie_string("a b", b"x") == ""
    assert H.cookie_string("k", b'a"b;c') == "k=abc"
    assert H.cookie_string("k", b"a b") == 'k="a b"'
    assert H._canon_header("content-type") == "Content-Type"
    assert H._canon_header("bad key") == "bad key"


def wrap_binary_body(body: bytes, name: str, typ: int, fid: int, seq: int) -> bytes:
    """thrift.WrapBinaryBody (thrift/binary.go): message header, the result
    field's header, the body, STOP."""
    nb = name.encode()
    return (struct.pack(">I", 0x80010000 | typ) + struct.pack(">i", len(nb)) + nb + struct.pack(">i", seq) +
            bytes([12]) + struct.pack(">h", fid) + body + b"\x00")


def test_http_conv(chk):
    """t2j.HTTPConv (conv/t2j/http_conv.go, ExampleHTTPConv_DoInto in
    conv/t2j/example_test.go:55-86): the REPLY of example3resp.bin; the body
    equals BinaryConv's with EnableHttpMapping, the headers and cookies are
    set, the raw body is the JSON. An EXCEPTION reply converts its field's
    type; a bad header or an unknown exception id errors."""
    import os
    g = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    fn = _example3_svc().functions()["ExampleMethod"]
    data = open(os.path.join(g, "example3resp.bin"), "rb").read()
    msg = wrap_binary_body(data, "ExampleMethod", t2j.REPLY, 0, 1)
    assert t2j.unwrap_binary_message(msg) == ("ExampleMethod", t2j.REPLY, 1, 0, data)
    opts = conv.Options(OmitHttpMappingErrors=True)
    hc = t2j.HTTPConv(H.ENCODING_THRIFT_BINARY, fn, conv=harness_conv(chk, opts))
    resp = H.HTTPResponse()
    buf = bytearray()
    hc.do_into(resp, msg, buf, opts)
    want_resp = H.HTTPResponse()
    want = harness_conv(chk, conv.Options(EnableHttpMapping=True, OmitHttpMappingErrors=True)).do(
        resp_desc("ExampleMethod"), data, want_resp)
    assert bytes(buf) == want and resp.body == want
    assert resp.headers["Heeader"] == want_resp.headers["Heeader"] and resp.cookies() == want_resp.cookies()
    # an exception reply: field 1 of the result (the declared exception)
    exc = fld(8, 1, struct.pack(">i", 400)) + fld(11, 255, tstr("boom")) + b"\x00"
    r2 = H.HTTPResponse()
    hc.do(r2, wrap_binary_body(exc, "ExampleMethod", t2j.EXCEPTION, 1, 2), opts)
    assert json.loads(r2.body) == {"code": 400, "msg": "boom"}
    with pytest.raises(H.ConvError) as ei:
        hc.do(H.HTTPResponse(), wrap_binary_body(exc, "ExampleMethod", t2j.EXCEPTION, 9, 2), opts)
    assert ei.value.behavior == "ErrUnknownField"
    with pytest.raises(H.ConvError) as ei:
        hc.do(H.HTTPResponse(), wrap_binary_body(data, "ExampleMethod", t2j.REPLY, 3, 1), opts)
    assert ei.value.behavior == "ErrInvalidParam"
    with pytest.raises(H.ConvError) as ei:
        hc.do(H.HTTPResponse(), b"\x00\x00\x00\x05hello", opts)
    assert ei.value.behavior == "ErrRead"
