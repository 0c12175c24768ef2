"""CPU: the host half of conv/j2t's HTTP mapping (dynamicgo_amd.http):
request getters (http/http.go), the text decoder writeStringValue uses
(thrift/binary.go:1176-1296 DecodeText, strconv semantics), handleHttpMappings
(conv/j2t/impl.go:243-292) and the Base writer (writeRequestBaseToThrift).
No GPU: nothing here converts a body."""
import math
import os
import struct

import pytest

from dynamicgo_amd import conv, http as H, thrift as T

IDL = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "idl")


def _nesting():
    return T.new_descriptor_from_path(os.path.join(IDL, "baseline.thrift")).functions()["NestingMethod"] \
        .request().struct.fields[0].type


def test_request_getters():
    r = conv.HTTPRequest(b'{"I32": 7, "s": "a\\nb", "o": {"x": [1, 2]}}', url="http://h:1/p?a=1&a=2&q=x%20y",
                         headers={"content-type": "application/json", "X-Key": "v"},
                         cookies={"c": "1"}, params={"id": "9"})
    assert r.get_header("x-key") == "v" and r.get_header("X-KEY") == "v" and r.get_header("nope") == ""
    assert r.get_query("a") == "1" and r.get_query("q") == "x y" and r.get_query("z") == ""
    assert r.get_cookie("c") == "1" and r.get_param("id") == "9" and r.get_host() == "h:1"
    # GetMapBody: raw JSON text of a member, strings unquoted (http/http.go:246-270)
    assert r.get_map_body("I32") == "7" and r.get_map_body("s") == "a\nb"
    assert r.get_map_body("o") == '{"x": [1, 2]}' and r.get_map_body("none") == ""
    f = conv.HTTPRequest(b"a=1&b=x+y", headers={"Content-Type": "application/x-www-form-urlencoded"})
    assert f.get_post_form("b") == "x y" and f.get_map_body("a") == "1"
    k = conv.HTTPRequest(b"", headers=[("Cookie", "u=1; v=2")])
    assert k.get_cookie("v") == "2"


def test_strconv_semantics():
    assert H.parse_int("+5") == 5 and H.parse_int("-9223372036854775808") == -2**63
    for bad in ("9223372036854775808", "1_0", "0x10", " 1", ""):
        with pytest.raises(ValueError):
            H.parse_int(bad)
    assert H.parse_float("0x1p3") == 8.0 and H.parse_float("-1.5e2") == -150.0 and H.parse_float(".5") == 0.5
    assert math.isinf(H.parse_float("-Inf")) and math.isnan(H.parse_float("NaN"))
    for bad in ("1_0", "1e400", "1.5f", " 1", "0x1"):
        with pytest.raises(ValueError):
            H.parse_float(bad)
    assert H.parse_bool("T") and not H.parse_bool("0")
    with pytest.raises(ValueError):
        H.parse_bool("yes")


def test_decode_text_known_answers():
    i32 = T.builtin("i32")
    assert H.decode_text("-2", i32, False, True) == struct.pack(">i", -2)
    assert H.decode_text("300", T.builtin("byte"), False, True) == bytes([300 & 0xFF])
    assert H.decode_text("1,2", T.list_of(i32), False, True) == bytes([8]) + struct.pack(">Iii", 2, 1, 2)
    assert H.decode_text("aGk=", T.TypeDescriptor(T.STRING, "binary"), False, True) == struct.pack(">I", 2) + b"hi"
    assert H.decode_text("aGk=", T.TypeDescriptor(T.STRING, "binary"), False, False) == struct.pack(">I", 4) + b"aGk="
    with pytest.raises(ValueError):
        H.decode_text("{}", T.map_of(T.builtin("string"), i32), False, True)  # non-JSON map text: not implemented
    assert H.is_json_string(' [1]') and H.is_json_string('"x"') and not H.is_json_string("[1") \
        and not H.is_json_string("   ")


def test_handle_http_mappings_nesting():
    sd = _nesting().struct
    req = conv.HTTPRequest(b"", url="http://x/y?ListI32=1,2", headers={"String": "hdr"},
                           cookies={"list_i64": "4"}, params={"double": "2.5"})
    hx = H.HMContext(conv.Options(EnableHttpMapping=True))
    b, mask, again = hx.handle_http_mappings(req, sd, False)
    # String (1, header), Double (3, path), ListI32 (5, query), ListI64 (13, cookie); I32 (4: http_code,
    # body) has no value: DEFAULT requireness without WriteDefaultField writes nothing but counts as set
    assert b == (bytes([11]) + struct.pack(">hI", 1, 3) + b"hdr" + bytes([4]) + struct.pack(">hd", 3, 2.5) +
                 bytes([15]) + struct.pack(">hBIii", 5, 8, 2, 1, 2) + bytes([15]) + struct.pack(">hBIq", 13, 10, 1, 4))
    order = [f.id for f in sorted(sd.fields, key=lambda f: f.id)]
    assert mask == sum(1 << order.index(i) for i in (1, 3, 4, 5, 13)) and not again
    # ReadHttpValueFallback: the missing one is read from the body instead (not in the mask)
    hx2 = H.HMContext(conv.Options(EnableHttpMapping=True, ReadHttpValueFallback=True))
    b2, mask2, again2 = hx2.handle_http_mappings(req, sd, False)
    assert b2 == b and mask2 == mask & ~(1 << order.index(4)) and again2 == {4: True}
    # WriteDefaultField: the missing DEFAULT field is written empty
    hx3 = H.HMContext(conv.Options(EnableHttpMapping=True, WriteDefaultField=True))
    b3, _, _ = hx3.handle_http_mappings(req, sd, False)
    k = b.index(bytes([15]) + struct.pack(">h", 5))  # ListI32 follows I32 in declaration order
    assert b3 == b[:k] + bytes([8]) + struct.pack(">hi", 4, 0) + b[k:]
    with pytest.raises(H.ConvError):
        H.HMContext(conv.Options(EnableHttpMapping=True)).handle_http_mappings(None, sd, False)


def test_base_writer():
    b = H.Base(Caller="caller", Extra={"key": "value"})
    t = b.thrift()
    s = lambda fid, v: bytes([11]) + struct.pack(">hI", fid, len(v)) + v  # noqa: E731
    assert t == (s(1, b"") + s(2, b"caller") + s(3, b"") + s(4, b"") + bytes([13]) + struct.pack(">h", 6) +
                 bytes([11, 11]) + struct.pack(">II", 1, 3) + b"key" + struct.pack(">I", 5) + b"value" + b"\x00")
    f = T.FieldDescriptor(255, "Base", T.struct_type("Base"), is_request_base=True)
    merged = []
    out, nw = H.write_request_base(b, f, b'{"Base":{"LogID":"2"}}', lambda jb, cb: merged.append(jb.LogID) or cb)
    assert nw and merged == ["2"] and out[:3] == bytes([12]) + struct.pack(">h", 255)
    out2, nw2 = H.write_request_base(b, f, b'{"Base":{"LogID":"2"}}', None)
    assert not nw2 and out2 == out


def _no_body_struct_desc():
    T.init_agw_annos()  # agw.source = "not_body_struct" -> api.no_body_struct (anno_mapping.go:125-126)
    svc = T.new_descriptor_from_path(os.path.join(IDL, "example3.thrift"), T.Options(use_default_value=True))
    return svc.functions()["NoBodyStructMethod"].request().struct.fields[0].type


NO_BODY_EXPECTED = (b"\x0c\x00\x01" + b"\x08\x00\x02" + struct.pack(">i", 1) +
                    b"\x08\x00\x03" + struct.pack(">i", 1) + b"\x00")


def test_no_body_struct_mapping():
    """apiNoBodyStruct.Request (http_mapping.go:299-344) as TestNoBodyStruct
    (conv/j2t/conv_test.go:1191-1212) drives it: B from the query, C (not in
    the request) its IDL default, A (unmapped) absent, then STOP, written as
    Thrift binary (Encoding ThriftBinary) after the field header."""
    td = _no_body_struct_desc()
    f = td.struct.field_by_id(1)
    assert f.http_mappings == [("api.no_body_struct", "NoBodyStruct")]
    req = conv.HTTPRequest(b"{}", url="http://localhost?b=1")
    hx = H.HMContext(conv.Options(EnableHttpMapping=True))
    b, mask, again = hx.handle_http_mappings(req, td.struct, False)
    assert b == NO_BODY_EXPECTED and mask == 1 and not again
