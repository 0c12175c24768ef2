"""Descriptor builders shared by the golden-vector generator and the tests.

Probe descriptors D1/D2/D3 follow SURVEY.md Appendix D; the others come from
the reference's testdata IDLs (copied into tests/golden/idl as data fixtures).
"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from dynamicgo_amd import thrift as T  # noqa: E402

IDL_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "idl")


def probe(variant: str) -> T.TypeDescriptor:
    """SURVEY.md Appendix D probe struct S (D1, D2, D3)."""
    a_type = T.builtin("i16") if variant == "D3" else T.builtin("i32")
    fields = [
        T.FieldDescriptor(1, "A", a_type, T.OPTIONAL, vm=T.VM_JSCONV if variant == "D3" else 0),
        T.FieldDescriptor(2, "B", T.builtin("string"), T.OPTIONAL),
        T.FieldDescriptor(3, "C", T.list_of(T.builtin("i64")), T.OPTIONAL),
        T.FieldDescriptor(4, "D", T.builtin("binary"), T.OPTIONAL),
        T.FieldDescriptor(5, "E", T.builtin("double"), T.OPTIONAL),
    ]
    if variant == "D2":
        fields[0].required = T.DEFAULT
        fields.append(T.FieldDescriptor(6, "M", T.map_of(T.builtin("i64"), T.builtin("string")), T.REQUIRED))
        fields.append(T.FieldDescriptor(7, "S", T.set_of(T.builtin("i64")), T.OPTIONAL))
    return T.struct_type("S", fields)


def vm_probe() -> T.TypeDescriptor:
    """D4: non-inline value mappings (agw.body_dynamic 257 and the reference
    tests' test.js_conv2 999, served by the host on ERR_VM_END) beside plain
    fields, at the root and in a nested struct."""
    from vm_maps import JSConv2, JS_CONV2
    bd, js2 = T.AgwBodyDynamic(), JSConv2()
    inner = T.struct_type("I", [
        T.FieldDescriptor(1, "x", T.builtin("string"), T.OPTIONAL, vm=T.VM_BODY_DYNAMIC, value_mapping=bd),
        T.FieldDescriptor(2, "y", T.builtin("i16"), T.REQUIRED, vm=JS_CONV2, value_mapping=js2),
        T.FieldDescriptor(3, "z", T.builtin("i32"), T.OPTIONAL),
    ])
    fields = [
        T.FieldDescriptor(1, "A", T.builtin("i32"), T.OPTIONAL, vm=JS_CONV2, value_mapping=js2),
        T.FieldDescriptor(2, "B", T.builtin("string"), T.OPTIONAL, vm=T.VM_BODY_DYNAMIC, value_mapping=bd),
        T.FieldDescriptor(3, "C", T.list_of(T.builtin("i64")), T.OPTIONAL),
        T.FieldDescriptor(4, "D", T.builtin("double"), T.OPTIONAL, vm=JS_CONV2, value_mapping=js2),
        T.FieldDescriptor(5, "E", T.builtin("i64"), T.OPTIONAL, vm=T.VM_BODY_DYNAMIC, value_mapping=bd),
        T.FieldDescriptor(6, "F", inner, T.OPTIONAL),
        T.FieldDescriptor(7, "G", T.list_of(inner), T.DEFAULT),
        T.FieldDescriptor(8, "H", T.builtin("string"), T.OPTIONAL, vm=T.VM_JSCONV),
    ]
    return T.struct_type("S4", fields)


def idl_desc(fname: str, method: str, opts=None) -> T.TypeDescriptor:
    svc = T.new_descriptor_from_path(os.path.join(IDL_DIR, fname), opts)
    return svc.functions()[method].request().struct.field_by_id(1).type \
        if svc.functions()[method].request().struct.field_by_id(1) else \
        svc.functions()[method].request().struct.fields[0].type
