"""CPU: host-side mirrors of the reference's Go layer (no GPU calls):
toFlags, the HTTPConv message header/footer, error explanation text."""
from dynamicgo_amd import conv


def test_to_flags_matches_reference():
    """toFlags conv/j2t/conv.go:98-127."""
    assert conv.to_flags(conv.Options()) == 0x1
    assert conv.to_flags(conv.Options(DisallowUnknownField=True)) == 0x0
    assert conv.to_flags(conv.Options(WriteDefaultField=True, EnableValueMapping=True)) == 0x7
    assert conv.to_flags(conv.Options(EnableHttpMapping=True, ReadHttpValueFallback=True)) == 0x109


def test_message_header_footer():
    """thrift.GetBinaryMessageHeaderAndFooter (thrift/binary.go:137-175)."""
    hdr, ftr = conv.get_binary_message_header_and_footer("ExampleMethod", conv.MSG_CALL, 1, 0)
    assert hdr == bytes.fromhex("80010001" "0000000d") + b"ExampleMethod" + bytes.fromhex("00000000" "0c0001")
    assert ftr == b"\x00"
    hdr, _ = conv.get_binary_message_header_and_footer("m", 2, 7, -1)
    assert hdr == bytes.fromhex("80010002" "00000001") + b"m" + bytes.fromhex("ffffffff" "0c0007")


def test_explain_native_error_texts():
    """explainNativeError (conv/j2t/impl_amd64.go:261-298) on hand-packed words."""
    src = b'{"UnknownField":"1"}'
    # ERR_UNKNOWN_FIELD at pos 15 (just past the key's closing quote), value = key length
    e = conv.J2TError(12 | (15 << 8) | (12 << 40), conv.explain_native_error(12 | (15 << 8) | (12 << 40), src))
    assert "unknown field 'UnknownField'" in str(e) and e.behavior == "ErrUnknownField"
    ret = 2 | (1 << 8) | ((ord("x") << 8 | 6) << 40)
    assert "invalid char 'x' for state J2T_OBJ_0" in conv.explain_native_error(ret, b"{xx}")
    ret = 9 | (0 << 8) | ((10 << 8 | 11) << 40)
    assert "expect type I64 but got type 11" in conv.explain_native_error(ret, b'"x"')
    assert "stack 4096 overflow" in conv.explain_native_error(7 | (4096 << 40), b"[")
    assert conv.J2TError(19, "").behavior == "ErrConvert"
