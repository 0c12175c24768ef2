"""CPU: non-inline value mapping (ERR_VM_END) in both checkers.

The reference FSM stops with ERR_VM_END at a value-mapped field
(native/thrift.c:641-665) and the Go host serves it (handleValueMapping,
conv/j2t/impl_amd64.go:117-155): oracle/ref_harness.c does that around the
reference's own j2t_fsm_exec, oracle/j2t_oracle.c inside its restatement
(oracle/vm_host.h). Here the two are checked against each other and against
TestAGWDynamicBody's expected values (conv/j2t/conv_test.go:922-946)."""
import random
import struct

import pytest

import fuzz
import oracle
import vm_maps
from dynamicgo_amd import thrift as T
from schemas import idl_desc, vm_probe

vm_maps.register()
F_VM = 0x5  # F_ALLOW_UNKNOWN | F_ENABLE_VM


def _checkers():
    ref = oracle.RefOracle()
    if ref is None:
        pytest.skip("oracle/_ref not built")
    return ref, oracle.PortOracle()


def dynamic_struct():
    return idl_desc("example3.thrift", "DynamicStructMethod")


def _tstr(b: bytes) -> bytes:
    return struct.pack(">I", len(b)) + b


def agw_dynamic_body_expected() -> bytes:
    """ExampleDynamicStruct{Query "1", JSON "[1,2,3]", InnerStruct{InnerJSON
    `{"a":"中文","b":1}`, Must "2"}} in the field order j2t writes it (JSON
    key order), as TestAGWDynamicBody's "no http-mapping" case decodes it."""
    inner = (b"\x0b\x00\x01" + _tstr('{"a":"中文","b":1}'.encode()) +
             b"\x0b\x00\x02" + _tstr(b"2") + b"\x00")
    return (b"\x0b\x00\x01" + _tstr(b"1") + b"\x0b\x00\x02" + _tstr(b"[1,2,3]") +
            b"\x0c\x00\x03" + inner + b"\x00")


AGW_DATA = '{"Query":"1","json":[1,2,3],"inner_struct":{"inner_json":{"a":"中文","b":1},"Must":"2"}}'.encode()
# conv.Options{EnableValueMapping, WriteRequireField, ReadHttpValueFallback} -> toFlags
AGW_FLAGS = 0x1 | 0x4 | 0x20 | 0x100


def test_agw_dynamic_body_checkers():
    ref, port = _checkers()
    fl = T.flatten(dynamic_struct())
    want = agw_dynamic_body_expected()
    assert ref.j2t(fl, AGW_DATA, AGW_FLAGS) == (0, want)
    assert port.j2t(fl, AGW_DATA, AGW_FLAGS) == (0, want)
    # without EnableValueMapping the array is a type error on a STRING field
    assert ref.j2t(fl, AGW_DATA, AGW_FLAGS & ~0x4)[0] & 0xFF == 13  # ERR_DISMATCH_TYPE2
    assert port.j2t(fl, AGW_DATA, AGW_FLAGS & ~0x4) == ref.j2t(fl, AGW_DATA, AGW_FLAGS & ~0x4)


VM_CASES = [
    b'{"B":{"k":[1,2]}}', b'{"B":"s"}', b'{"B": 12 }', b'{"A":"7","D":"1.5"}', b'{"A":7,"D":-2e3}',
    b'{"A":"x"}', b'{"A":99999999999999999999}', b'{"E":1}', b'{"F":{"x":[true],"y":"3"}}',
    b'{"F":{"z":1}}', b'{"G":[{"y":1},{"y":"2","x":null}]}', b'{"B":[1', b'{"B":1}', b'{"B":null}',
    b'{"A":1.5}', b'{"D":"abc"}', b'{"H":"5","A":3}', b'{"B":"\\u00e9\\n"}', b'{"B":1,"B":2,"B":3}',
]


@pytest.mark.parametrize("flags", [0x5, 0x1, 0x25, 0x7])
def test_vm_cases(flags):
    ref, port = _checkers()
    fl = T.flatten(vm_probe())
    for m in VM_CASES:
        assert ref.j2t(fl, m, flags) == port.j2t(fl, m, flags), (m, flags)


def vm_message(rng) -> bytes:
    """A D4 message whose value-mapped fields mostly convert: int / decimal
    text (quoted or bare) on the test.js_conv2 fields, any JSON value on the
    body_dynamic ones, the nested struct's required y present."""
    def num(i):
        v = str(rng.randint(-2**40, 2**40)) if i else rng.choice(["1.5", "-0.25", "3e5", "7", "-1E-3", "0.1"])
        return '"%s"' % v if rng.random() < 0.5 else v

    def inner():
        it = ['"y":' + num(True)]
        if rng.random() < 0.7:
            it.append('"x":' + fuzz.gen_any(rng))
        if rng.random() < 0.3:
            it.append('"z":%d' % rng.randint(-5, 5))
        rng.shuffle(it)
        return "{" + ",".join(it) + "}"

    items = []
    for _ in range(rng.randint(1, 7)):
        k = rng.choice("ABCDFGH")
        v = {"A": lambda: num(True), "B": lambda: fuzz.gen_any(rng), "C": lambda: "[1,2]",
             "D": lambda: num(False), "F": inner, "G": lambda: "[" + ",".join(inner() for _ in range(rng.randint(0, 3))) + "]",
             "H": lambda: '"9"'}[k]()
        items.append('"%s":%s' % (k, v))
    return fuzz.spacify(rng, "{" + ",".join(items) + "}").encode()


def test_vm_targeted():
    ref, port = _checkers()
    rng = random.Random(5)
    fl = T.flatten(vm_probe())
    ok = 0
    for _ in range(800):
        m = vm_message(rng)
        r = ref.j2t(fl, m, 0x5)
        assert r == port.j2t(fl, m, 0x5), m
        ok += r[0] == 0
    assert ok > 400  # mostly served callbacks, not errors


def test_vm_fuzz():
    ref, port = _checkers()
    rng = random.Random(77)
    for td in (vm_probe(), dynamic_struct()):
        fl = T.flatten(td)
        for _ in range(600):
            m = fuzz.gen_message(rng, td)
            flags = rng.choice([0x5, 0x7, 0x25, 0x1])
            assert ref.j2t(fl, m, flags) == port.j2t(fl, m, flags), (m, flags)
