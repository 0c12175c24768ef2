"""GPU: the reference's HTTP-mapping callbacks served around the GPU
conversion (BinaryConv.do_batch_http).

The host restates handleHttpMappings / writeStringValue (dynamicgo_amd.http);
the GPU writes each struct's entry wherever the reference raises ERR_HM and
hands the root's ERR_HM_END back (DG_ST_HM_END). The checker is the
reference's own FSM (oracle/_ref, native.c) driven by the same host entries
at each ERR_HM (dgref_j2t_hm3) and finished by the same handleUnmatchedFields
restatement at the root's ERR_HM_END: the bodies, the resume points, the
requires masks and the field caches are the reference's."""
import json
import os
import random
import struct
import zlib

import pytest

import oracle
from dynamicgo_amd import conv, http as H, thrift as T, workloads as W

pytestmark = pytest.mark.gpu
IDL = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "idl")
REF = oracle.RefOracle()


def _req_type(path, method, opts=None):
    svc = T.new_descriptor_from_path(os.path.join(IDL, path), opts)
    return svc.functions()[method].request().struct.fields[0].type


def _entries(flat, hx, req):
    out = []
    for sd in flat.structs:
        if not sd.hms:
            out.append((b"", 0))
            continue
        try:
            b, m, _ = hx.handle_http_mappings(req, sd, False)
            out.append((b, m))
        except H.ConvError:
            out.append(None)
    return out


def _expected(td, body, req, opts):
    """(kind, value): ("ok", bytes) or ("err", code or ConvError type)."""
    flat = T.flatten(td)
    hx = H.HMContext(opts, conv.BinaryConv(opts)._nested(conv.to_flags(opts)))
    if len(body) == 0:
        try:
            return "ok", hx.empty_body(req, td.struct)
        except H.ConvError as e:
            return "err", e.behavior
    ents = _entries(flat, hx, req)

    def nested_end(si, ids):  # a nested struct's ERR_HM_END: handleUnmatchedFields (top = true) + STOP
        try:
            return hx.handle_unmatched_fields(req, flat.structs[si], ids, True) + b"\x00"
        except H.ConvError:
            return None
    REF.set_hm_end_cb(nested_end)
    try:
        r, out, fc = REF.j2t_hm3(flat, body, conv.to_flags(opts), ents)
    finally:
        REF.set_hm_end_cb(None)
    if r == 0:
        return "ok", out
    if r & 0xFF == 21:  # the root's ERR_HM_END: handleUnmatchedFields + STOP
        try:
            return "ok", out + hx.handle_unmatched_fields(req, td.struct, fc, True) + b"\x00"
        except H.ConvError as e:
            return "err", e.behavior
    if r & 0xFF == 19:  # ERR_HM where the host failed for that struct
        return "err", "host"
    return "err", r


def _check(td, bodies, reqs, opts):
    outs, errs = conv.BinaryConv(opts).do_batch_http(td, bodies, reqs)
    n_ok = 0
    for b, q, o, e in zip(bodies, reqs, outs, errs):
        kind, v = _expected(td, b, q, opts)
        if kind == "ok":
            assert e is None, (b[:120], e)
            assert o == v, b[:120]
            n_ok += 1
        elif v == "host" or isinstance(v, str):
            assert isinstance(e, H.ConvError), (b[:120], e)
        else:
            assert isinstance(e, conv.J2TError) and e.ret == v, (b[:120], e, v)
    return n_ok


def _nesting_req(rng, body):
    kw = {"headers": {"Content-Type": "application/json"}, "cookies": {}, "params": {}}
    q = []
    if rng.random() < 0.8:
        kw["headers"]["String"] = "h%d" % rng.randint(0, 999)
    if rng.random() < 0.7:
        kw["params"]["double"] = rng.choice(["2.5", "-1e3", "0x1p4", "7"])
    if rng.random() < 0.7:
        q.append("ListI32=" + ",".join(str(rng.randint(-9, 9)) for _ in range(rng.randint(1, 4))))
    if rng.random() < 0.7:
        kw["cookies"]["list_i64"] = ",".join(str(rng.randint(-2**40, 2**40)) for _ in range(rng.randint(1, 3)))
    if rng.random() < 0.1:
        kw["params"]["double"] = "not-a-number"  # writeStringValue fails: ErrConvert
    return conv.HTTPRequest(body, url="http://gw/nesting?" + "&".join(q), **kw)


@pytest.mark.parametrize("optname", ["default", "write_default", "fallback", "fallback_traceback", "write_require"])
def test_nesting_requests_vs_reference_fsm(optname):
    """Nesting (baseline.thrift): header / path / query / cookie / body mapped
    root fields, with random requests and bodies (some with the mapped keys
    present, some empty, null or malformed)."""
    opts = {"default": conv.Options(EnableHttpMapping=True),
            "write_default": conv.Options(EnableHttpMapping=True, WriteDefaultField=True),
            "fallback": conv.Options(EnableHttpMapping=True, ReadHttpValueFallback=True),
            "fallback_traceback": conv.Options(EnableHttpMapping=True, ReadHttpValueFallback=True,
                                               TracebackRequredOrRootFields=True),
            "write_require": conv.Options(EnableHttpMapping=True, WriteRequireField=True)}[optname]
    td = _req_type("baseline.thrift", "NestingMethod")
    rng = random.Random(zlib.crc32(optname.encode()))
    bodies = []
    for k in range(300):
        o = json.loads(W.nesting_obj(rng))
        for key in list(o):
            if rng.random() < 0.3:
                del o[key]
        bodies.append(json.dumps(o).encode())
    bodies += [b"", b"{}", b"null", b"{]", b'{"I32":1,"String":"body"}', b"[]"]
    reqs = [_nesting_req(rng, b) for b in bodies]
    assert _check(td, bodies, reqs, opts) > 250


def test_example3_http2thrift():
    """conv/j2t/conv_test.go:169-188 (TestConvHTTP2Thrift) with the request of
    getExampleReq(setIs=true) (conv_test.go:255-296): mapped fields of the root
    AND of every nested InnerBase (root, list element, map value). Checked
    against the reference FSM and, like the Go test, on the decoded values."""
    td = _req_type("example3.thrift", "ExampleMethod")
    body = open(os.path.join(os.path.dirname(IDL), "example3req.json"), "rb").read()
    url = "http://localhost:8888/root?inner_query=abcd&query=1%2C2%2C3"  # url.Values.Encode: sorted keys
    req = conv.HTTPRequest(body, url=url, headers={"Content-Type": "application/json", "heeader": "true",
                                                   "inner_string": "abcd"},
                           cookies={"cookie": "-1.00001"}, params={"path": "<>"})
    opts = conv.Options(EnableHttpMapping=True)
    assert _check(td, [body], [req], opts) == 1
    out = conv.BinaryConv(opts).do(td, body, req=req)
    from dynamicgo_amd import t2j
    js = json.loads(t2j.BinaryConv(conv.Options()).do(td, out))
    exp = json.loads(body)
    assert js["Path"] == "<>" and js["Query"] == ["1", "2", "3"] and js["Header"] is True
    assert js["Cookie"] == -1.00001 and js["RawUri"] == url and js["msg"] == exp["msg"]
    ib = js["InnerBase"]
    assert ib["String"] == "abcd" and ib["InnerQuery"] == "abcd"
    assert ib["ListInnerBase"][0]["String"] == "abcd" and ib["ListInnerBase"][0]["InnerQuery"] == "abcd"
    assert ib["MapStringInnerBase"]["innerx"]["String"] == "abcd"
    assert ib["Int64"] == exp["InnerBase"]["Int64"] and ib["MapInt32String"] == exp["InnerBase"]["MapInt32String"]


def test_httpconv_do_batch_frames_mapped_requests():
    """HTTPConv.do_batch for a method whose root has mapped fields: the host
    half, then the message header/footer (http_conv.go:68-94)."""
    fn = T.new_descriptor_from_path(os.path.join(IDL, "baseline.thrift")).functions()["NestingMethod"]
    hc = conv.HTTPConv(conv.ENCODING_THRIFT_BINARY, fn)
    rng = random.Random(3)
    bodies = W.gen_nested_batch(rng, 200) + [b""]
    reqs = [_nesting_req(rng, b) for b in bodies]
    outs, errs = hc.do_batch(reqs)
    opts = conv.Options(EnableHttpMapping=True)
    for b, q, o, e in zip(bodies, reqs, outs, errs):
        kind, v = _expected(hc.st, b, q, opts)
        if kind == "ok":
            assert e is None and o == hc.top + v + hc.bottom
        else:
            assert e is not None and o == b""


def test_thrift_request_base():
    """TestThriftRequestBase / TestMergeBase (conv/j2t/conv_test.go:620-672,
    1264-1330): the context Base written first (writeRequestBaseToThrift);
    with a JSON Base and MergeBaseFunc the merged one, the body's skipped
    (F_NO_WRITE_BASE)."""
    topts = T.Options(enable_thrift_base=True)
    td = _req_type("example3.thrift", "ExampleMethod", topts)
    data = json.loads(open(os.path.join(os.path.dirname(IDL), "example3req.json")).read())
    base = H.Base(Caller="caller", Extra={"key": "value"})
    from dynamicgo_amd import t2j

    def decode(b):
        return json.loads(t2j.BinaryConv(conv.Options()).do(td, b))

    nob = dict(data)
    nob.pop("Base", None)
    opts = conv.Options(EnableThriftBase=True, WriteDefaultField=True)
    out = conv.BinaryConv(opts).do(td, json.dumps(nob).encode(), base=base)
    rb = next(f for f in td.struct.fields if f.is_request_base)
    assert out.startswith(H.field_begin(rb) + base.thrift())
    assert decode(out)["Base"]["Caller"] == "caller" and decode(out)["Base"]["Extra"] == {"key": "value"}
    # ctx + json base, no merge func: both written, the body's last (it wins on decode)
    out2 = conv.BinaryConv(opts).do(td, json.dumps(data).encode(), base=base)
    assert decode(out2)["Base"]["LogID"] == data["Base"]["LogID"]

    def merge(frm, to):
        frm.LogID, frm.Caller, frm.Addr, frm.Client, frm.TrafficEnv = to.LogID, to.Caller, to.Addr, to.Client, \
            to.TrafficEnv
        if to.Extra is not None:
            frm.Extra = dict(frm.Extra or {}, **to.Extra)
        return frm
    d3 = dict(data, Base={"LogID": "2", "Client": "2", "Extra": {"a": "2", "c": "2"}})
    opts3 = conv.Options(EnableThriftBase=True, MergeBaseFunc=merge)
    out3 = conv.BinaryConv(opts3).do(td, json.dumps(d3).encode(), base=H.Base(LogID="1", Extra={"a": "1", "b": "1"}))
    got = decode(out3)["Base"]
    assert got["LogID"] == "1" and got["Client"] == "" and got["Extra"] == {"a": "1", "b": "1", "c": "2"}


def test_no_body_struct():
    """TestNoBodyStruct (conv/j2t/conv_test.go:1191-1212): the whole Do."""
    from test_http_host import NO_BODY_EXPECTED, _no_body_struct_desc
    td = _no_body_struct_desc()
    req = conv.HTTPRequest(b"{}", url="http://localhost?b=1")
    out = conv.BinaryConv(conv.Options(EnableHttpMapping=True)).do(td, b"{}", req=req)
    assert out == NO_BODY_EXPECTED + b"\x00"
    assert _check(td, [b"{}", b'{"NoBodyStruct":{"A":5}}'], [req, req], conv.Options(EnableHttpMapping=True)) == 2
