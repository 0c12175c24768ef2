"""Error-text parity: the reference's own error-path assertions
(conv/j2t/conv_amd64_test.go:44-180, TestError) on ret words produced by the
GPU, explained by conv.explain_native_error (the restatement of
explainNativeError, conv/j2t/impl_amd64.go:261-298). The packed word itself
must also equal the oracle's."""
import json
import os

import pytest

import oracle
from dynamicgo_amd import conv, thrift as T
from schemas import idl_desc

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _check(td, data, opts, behavior, substr):
    cv = conv.BinaryConv(opts)
    with pytest.raises(conv.J2TError) as ei:
        cv.do(td, data)
    e = ei.value
    chk = oracle.RefOracle() or oracle.PortOracle()
    er, _ = chk.j2t(T.flatten(td), data, conv.to_flags(opts))
    assert e.ret == er, (hex(e.ret), hex(er))
    assert e.behavior == behavior, e.behavior
    assert substr in str(e), str(e)
    return e


def example():
    return idl_desc("example3.thrift", "ExampleMethod")


def test_err_null_required():
    td = idl_desc("null.thrift", "NullTest")
    data = open(os.path.join(GOLDEN, "null_err.json"), "rb").read()
    _check(td, data, conv.Options(), "ErrMissRequiredField", "missing required field 3")
    out = conv.BinaryConv(conv.Options(WriteRequireField=True)).do(td, data)
    assert out  # WriteRequireField: no error


def test_invalid_char():
    _check(example(), b"{xx}", conv.Options(), "ErrRead", "invalid char 'x' for state J2T_OBJ_0")


def test_invalid_number_fmt():
    td = idl_desc("example3.thrift", "Int2FloatMethod")
    _check(td, b'{"Float64":1.x1}', conv.Options(EnableValueMapping=True), "ErrConvert", "unexpected number type")


def test_unsupported_thrift_type():
    td = idl_desc("example3.thrift", "ErrorMethod")
    _check(td, b'{"MapInnerBaseInnerBase":{"a":"a"}', conv.Options(), "ErrUnsupportedType",
           "unsupported thrift type STRUCT")


def test_dismatch_type():
    d = json.loads(open(os.path.join(GOLDEN, "example3req.json"), "rb").read())
    d["code_code"] = "1.1"
    data = json.dumps(d, ensure_ascii=False, separators=(",", ":")).encode()
    _check(example(), data, conv.Options(), "ErrDismatchType", "expect type I64 but got type 11")


def test_unknown_field():
    td = idl_desc("example3.thrift", "ErrorMethod")
    _check(td, b'{"UnknownField":"1"}', conv.Options(DisallowUnknownField=True), "ErrUnknownField",
           "unknown field 'UnknownField'")


def test_decode_base64():
    td = idl_desc("example3.thrift", "ErrorMethod")
    _check(td, b'{"Base64":"xxx"}', conv.Options(), "ErrRead", "decode base64 error: ")


def test_recurse_exceed_max():
    """The reference reaches ERR_RECURSE_MAX through MockConv's preset stack
    pointer; here through real nesting past MAX_RECURSE (4096): the 4096th
    push fails with the stack depth as the value."""
    deep = T.TypeDescriptor(T.LIST, "list")
    deep.elem = deep  # list<list<...>>, a cyclic descriptor (cycles are allowed, SelfRef)
    e = _check(deep, b"[" * 4200 + b"]" * 4200, conv.Options(), "ErrStackOverflow", "stack 4096 overflow")
    assert e.code == 7


# ---- HTTP-mapping pre-split (DG_F_HM_SPLIT) ----
HM, HM_SPLIT = 0x8, 1 << 20


@pytest.mark.parametrize("method,flags", [("NestingMethod", 0x1), ("NestingMethod", 0x7), ("NestingMethod", 0x83),
                                          ("Nesting2Method", 0x1)])
def test_hm_split_vs_reference(method, flags):
    """The root struct's HTTP-mapped fields written by the host (the prefix),
    the body converted on the GPU: prefix + GPU bytes == the reference FSM
    resumed after handleHttpMappings (mapped keys in the body skipped, mapped
    fields counted as set). Nested mapped structs still return ERR_HM."""
    import random
    import fuzz
    from schemas import idl_desc
    from test_gpu_parity import _raw_batch
    ref = oracle.RefOracle()
    if ref is None:
        pytest.skip("oracle/_ref not built")
    td = idl_desc("baseline.thrift", method)
    fl = T.flatten(td)
    rng = random.Random(77 + flags)
    msgs = [fuzz.gen_message(rng, td, mutate_p=rng.random() < 0.3) for _ in range(400)]
    prefix = b"\x0b\x00\x01\x00\x00\x00\x02hm" + b"\x08\x00\x04\x00\x00\x00\x07"
    outs, rets = _raw_batch(fl, msgs, flags | HM | HM_SPLIT)
    # the host writes a prefix only when the root struct has mapped fields and
    # the body is a struct (a null body converts to nothing)
    root_hm = any(f.http_mappings for f in td.struct.fields)
    bad = []
    for i, m in enumerate(msgs):
        if not m:  # an empty body is the Go prelude's (handleHttpMappings with nobody=true, impl.go:52-82)
            continue
        er, eo = ref.j2t_hm(fl, m, flags | HM, prefix)
        got = (prefix if root_hm else b"") + outs[i] if int(rets[i]) == 0 and outs[i] else b""
        if int(rets[i]) != er or got != eo:
            bad.append((m[:80], hex(int(rets[i])), hex(er), got[:40], eo[:40]))
    assert not bad, bad[:4]
