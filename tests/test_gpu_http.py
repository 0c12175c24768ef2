"""HTTPConv (conv/j2t/http_conv.go:28-114) on the GPU: the message header and
footer (thrift.GetBinaryMessageHeaderAndFooter, thrift/binary.go:137-175)
around the body converted with EnableHttpMapping, framed by
dg_pack_device_framed. Bodies are checked against the oracle with the same
flags; structs with HTTP-mapped fields return the reference's ERR_HM code
(the Go host's callback, out of scope)."""
import os
import random

import pytest

import oracle
from dynamicgo_amd import conv, thrift as T, workloads as W

pytestmark = pytest.mark.gpu
IDL = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "idl")


def fn(method):
    return T.new_descriptor_from_path(os.path.join(IDL, "baseline.thrift")).functions()[method]


def test_header_footer_known_answer():
    hdr, ftr = conv.get_binary_message_header_and_footer("SimpleMethod", conv.MSG_CALL, 1, 0)
    assert hdr.hex() == "80010001" + "0000000c" + b"SimpleMethod".hex() + "00000000" + "0c0001"
    assert ftr == b"\x00"


def test_httpconv_do_vs_oracle():
    hc = conv.HTTPConv(conv.ENCODING_THRIFT_BINARY, fn("SimpleMethod"))
    chk = oracle.RefOracle() or oracle.PortOracle()
    fl = T.flatten(hc.st)
    flags = conv.to_flags(conv.Options(EnableHttpMapping=True))
    for body in [W.c1_simple_json(), b"{}", b"", b'{"I32Field":7}']:
        out = hc.do(conv.HTTPRequest(body))
        er, eo = chk.j2t(fl, body, flags)
        assert er == 0
        assert out == hc.top + eo + hc.bottom
        buf = bytearray(b"xy")
        hc.do_into(conv.HTTPRequest(body), buf)
        assert bytes(buf) == b"xy" + out


def test_httpconv_batch_framed_on_gpu():
    """A root without HTTP-mapped fields: converted and framed on the GPU
    (dg_pack_device_framed), or, with an empty body in the batch, through the
    host half (the empty-body branch, conv/j2t/impl.go:52-82). Roots with
    mapped fields: tests/test_gpu_http_map.py."""
    rng = random.Random(5)
    chk = oracle.RefOracle() or oracle.PortOracle()
    hc = conv.HTTPConv(conv.ENCODING_THRIFT_BINARY, fn("SimpleMethod"))
    fl = T.flatten(hc.st)
    flat_bodies = W.gen_flat_batch(rng, 3000)
    for bodies in (flat_bodies + [b"{]", b"{}", b'{"I32Field":tru}'], flat_bodies[:500] + [b""]):
        reqs = [conv.HTTPRequest(b) for b in bodies]
        for opts in (conv.Options(), conv.Options(WriteDefaultField=True)):
            outs, errs = hc.do_batch(reqs, opts)
            flags = conv.to_flags(opts) | conv.F_HTTP_MAPPING
            for b, o, e in zip(bodies, outs, errs):
                er, eo = chk.j2t(fl, b, flags)
                assert (e.ret if e is not None else 0) == er, b[:80]
                assert o == (hc.top + eo + hc.bottom if er == 0 else b""), b[:80]


def test_do_batch_hm_split_mirror():
    """BinaryConv.do_batch_hm_split: the Python mirror of the pre-split flow
    (prefix from the host + GPU body) equals the resumed reference."""
    import oracle
    from schemas import idl_desc
    ref = oracle.RefOracle()
    if ref is None:
        pytest.skip("oracle/_ref not built")
    td = idl_desc("baseline.thrift", "NestingMethod")
    fl = T.flatten(td)
    bodies = [b'{"String":"x","I64":5,"ListString":["a"],"Double":1.5}', b'{}', b'{"I32":7,"Byte":1}', b'{"I64":']
    prefixes = [b"\x0b\x00\x01\x00\x00\x00\x01h", b"", b"\x04\x00\x03" + bytes(8), b"\x08\x00\x04\x00\x00\x00\x01"]
    outs, rets = conv.BinaryConv(conv.Options()).do_batch_hm_split(td, bodies, prefixes)
    for b, p, o, r in zip(bodies, prefixes, outs, rets):
        er, eo = ref.j2t_hm(fl, b, 0x1 | 0x8, p)
        assert (int(r), o) == (er, eo)
