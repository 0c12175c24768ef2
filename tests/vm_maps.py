"""Value mappings the tests register (the Python side of oracle/vm_host.h).

``JSConv2`` restates apiJSConv2.Write (thrift/annotation/value_mapping_test.go:
82-111), the non-inline value mapping (type 999, "test.js_conv2") the
reference's own tests register. strconv.ParseInt / ParseFloat are restricted
to plain decimal text exactly as oracle/vm_host.h restricts them, so the GPU
path (which calls this on ERR_VM_END) and both CPU checkers agree.
"""
import re
import struct

from dynamicgo_amd import thrift as T

JS_CONV2 = 999
_INT = re.compile(rb"[+-]?[0-9]+\Z")
_FLOAT = re.compile(rb"[+-]?([0-9]+(\.[0-9]*)?|\.[0-9]+)([eE][+-]?[0-9]+)?\Z")


class JSConv2(T.ValueMapping):
    def write(self, field, src: bytes) -> bytes:
        if not src:
            raise T.ValueMappingError("empty value")
        if src[:1] == b'"':
            if len(src) < 2:
                raise T.ValueMappingError("bad quote")
            src = src[1:-1]
        t = field.type.type
        if t in (T.BYTE, T.I16, T.I32, T.I64):
            if not _INT.match(src):
                raise T.ValueMappingError("invalid syntax")
            v = int(src)
            if not -2**63 <= v < 2**63:
                raise T.ValueMappingError("value out of range")
            n = {T.BYTE: 1, T.I16: 2, T.I32: 4, T.I64: 8}[t]
            return (v & ((1 << (8 * n)) - 1)).to_bytes(n, "big")  # BinaryProtocol.WriteInt truncation
        if t == T.DOUBLE:
            if not _FLOAT.match(src):
                raise T.ValueMappingError("invalid syntax")
            v = float(src)
            if v in (float("inf"), float("-inf")):
                raise T.ValueMappingError("value out of range")
            return struct.pack(">d", v)
        raise T.ValueMappingError("unsupported type %d" % t)


def register():
    """thrift.RegisterAnnotation(..., "test.js_conv2") + InitAGWAnnos."""
    T.register_value_mapping("test.js_conv2", JS_CONV2, JSConv2())
    T.init_agw_annos()
