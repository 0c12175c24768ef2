"""Generate tests/golden/j2t_golden.jsonl and descs.json from the REFERENCE
engine (oracle/_ref/libdgref.so = /root/reference/native/native.c compiled by
oracle/Makefile). Run in the build container (needs /root/reference once):

    make -C oracle ref && python tests/golden/gen_golden.py

Each row: {"desc": name, "flags": int, "json": hex, "ret": int, "out": hex}.
The rows are data (inputs + the reference's outputs); descs.json holds the
flattened dg_desc v1 blobs they refer to.
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), HERE]

import oracle  # noqa: E402
import fuzz  # noqa: E402
from dynamicgo_amd import thrift as T, workloads as W  # noqa: E402
from schemas import idl_desc, probe  # noqa: E402


def descriptors():
    d = {
        "D1": probe("D1"), "D2": probe("D2"), "D3": probe("D3"),
        "simple": idl_desc("baseline.thrift", "SimpleMethod"),
        "nesting": idl_desc("baseline.thrift", "NestingMethod"),
        "nesting2": idl_desc("baseline.thrift", "Nesting2Method"),
        "example3": idl_desc("example3.thrift", "ExampleMethod"),
        "example3_dflt": idl_desc("example3.thrift", "ExampleMethod", T.Options(use_default_value=True)),
        "null": idl_desc("null.thrift", "NullTest"),
        "string_root": T.builtin("string"),
        "i64_root": T.builtin("i64"),
        "large": W.large_desc(),
        "nesting_i64": W.nesting_i64_desc(),
    }
    return d


APPENDIX_D = [
    ("D1", 0x1, b'{"A":-12,"B":"h\\u00e9llo","C":[1,2,null,3],"D":"/////w==","E":1.5e-3}'),
    ("D1", 0x1, b'{"A":1.9,"C":[],"B":"x","Z":{"q":[1,{"a":2}]},"E":-0}'),
    ("D1", 0x1, b'{"D":"xxx"}'), ("D1", 0x1, b'{"A":01}'), ("D1", 0x11, b'{"A":1} xyz'),
    ("D1", 0x11, b'{"A":1,"A":2}'), ("D1", 0x11, b'{"B":"a\tb\\u0000"}'), ("D1", 0x11, b'{"E":1e400}'),
    ("D1", 0x11, b'{"C":[99999999999999999999]}'), ("D1", 0x11, b'{"C":[-]}'), ("D1", 0x11, b'{"A":"12"}'),
    ("D1", 0x11, b'{"E":"1.5"}'), ("D1", 0x11, b'{"C":[1.0e2, -9223372036854775808, 9223372036854775808]}'),
    ("D1", 0x11, b'{"D":"aGk=\\n"}'), ("D1", 0x11, b'{"D":"aGk"}'), ("D1", 0x11, b'{"B":"\\ud800"}'),
    ("D1", 0x11, b'{"E":0.1}'), ("D1", 0x11, b'{"E":123456789012345678901234567890e-10}'),
    ("D2", 0x1, b'{"M":{"12abc":"x","-3":"y"}}'), ("D2", 0x1, b'{"M":{"":"x"}}'),
    ("D2", 0x1, b'{"M":{"1":null,"2":"z"}}'), ("D2", 0x1, b'{"A":5}'), ("D2", 0x1, b'{"M":{}}'),
    ("D2", 0x1, b'{"S":[1,2],"M":{}}'), ("D2", 0x23, b'{"B":"k"}'),
    ("D3", 0x5, b'{"A":"7"}'), ("D3", 0x5, b'{"A":7}'), ("D3", 0x5, b'{"A":""}'),
]


def nesting_payload():
    """baseline.Nesting sample (listCount = mapCount = 16), keys sorted like encoding/json."""
    simple = W.c1_simple_json().decode()
    s = W.go_json_string("你好,\b\n\r\t世界" * 2)
    import base64
    b = base64.b64encode(bytes(range(16)) * 2).decode()
    keys = sorted(str(i) for i in range(16))
    return ('{"String":%s,"ListSimple":[%s],"Double":1.7976931348623157e+308,"I32":2147483647,'
            '"ListI32":[%s],"I64":9223372036854775807,"MapStringString":{%s},"SimpleStruct":%s,'
            '"MapI32I64":{%s},"ListString":[%s],"Binary":"%s","MapI64String":{%s},"ListI64":[%s],'
            '"Byte":127,"MapStringSimple":{%s}}' % (
                s, ",".join([simple] * 16), ",".join(["-2147483648"] * 16),
                ",".join('"%s":%s' % (k, s) for k in keys), simple,
                ",".join('"%s":-9223372036854775808' % k for k in keys), ",".join([s] * 16), b,
                ",".join('"%s":%s' % (k, s) for k in keys), ",".join(["-9223372036854775808"] * 16),
                ",".join('"%s":%s' % (k, simple) for k in keys))).encode()


def main():
    ref = oracle.RefOracle()
    if ref is None:
        sys.exit("oracle/_ref not built: make -C oracle ref")
    descs = descriptors()
    flats = {k: T.flatten(v) for k, v in descs.items()}
    rows = []

    def add(name, flags, js):
        r, out = ref.j2t(flats[name], js, flags)
        rows.append({"desc": name, "flags": flags, "json": js.hex(), "ret": r, "out": out.hex()})

    for name, fl, js in APPENDIX_D:
        add(name, fl, js)
    # TestSimpleArgs conv/j2t/conv_test.go:1214-1246
    add("string_root", 1, b'"hello"')
    add("string_root", 1, b"hel\\lo")
    add("i64_root", 1, b"9223372036854775807")
    add("simple", 1, W.c1_simple_json())
    add("simple", 1 | 2 | 4, W.c1_simple_json())
    add("nesting", 1, nesting_payload())
    ex3 = open(os.path.join(HERE, "example3req.json"), "rb").read()
    for fl in (1, 0, 2, 0x20, 0x80, 0x4, 0x10, 0x40, 0x200):
        add("example3", fl, ex3)
        add("example3_dflt", fl | 2, ex3)
    for fn in ("null_pass.json", "null_err.json"):
        add("null", 1, open(os.path.join(HERE, fn), "rb").read())
    add("simple", 1, b"")
    add("simple", 1, b"null")
    add("simple", 1, b"   {}   ")
    add("simple", 0, b'{"Unknown":1}')
    # depth: nested unknown values and deep lists
    add("D1", 1, b'{"Z":' + b"[" * 100 + b"]" * 100 + b"}")
    add("D1", 1, b'{"Z":' + b"[" * 5000 + b"]" * 5000 + b"}")
    deepd = T.list_of(T.builtin("i64"))
    for _ in range(40):
        deepd = T.list_of(deepd)
    flats["deep_list"] = T.flatten(deepd)
    add("deep_list", 1, b"[" * 41 + b"[1,2]" + b"]" * 41)
    # fuzz rows
    rng = random.Random(20261015)
    FLAGS = [0x1, 0x0, 0x11, 0x5, 0x23, 0x41, 0x83, 0xf7, 0x15, 0x2, 0x20, 0x80, 0x100, 0x201]
    for name in ("D1", "D2", "D3", "simple", "nesting", "example3", "null", "nesting2"):
        for _ in range(250):
            add(name, rng.choice(FLAGS), fuzz.gen_message(rng, descs[name]))
    # F_ENABLE_HM (0x8) and F_ENABLE_HM|F_TRACE_BACK (0x108): structs with
    # HTTP-mapped fields return ERR_HM at entry (native/thrift.c:1119-1123),
    # unset tracked fields ERR_HM_END at '}' (native/thrift.c:898-903,
    # 952-957), mapped keys are skipped (native/thrift.c:725); the callbacks
    # themselves are the Go host's (out of scope), the codes are the parity bar
    hm_rng = random.Random(20261016)
    HM_FLAGS = [0x8, 0x9, 0x108, 0x109, 0x10b, 0x12b, 0x18f]
    for name in ("simple", "nesting", "nesting2", "example3", "null", "D1", "D2"):
        for _ in range(60):
            add(name, hm_rng.choice(HM_FLAGS), fuzz.gen_message(hm_rng, descs[name]))
    for fl in HM_FLAGS:
        add("nesting", fl, nesting_payload())
        add("simple", fl, W.c1_simple_json())
        add("example3", fl, ex3)
    with open(os.path.join(HERE, "j2t_golden.jsonl"), "w") as fh:
        for r in rows:
            fh.write(json.dumps(r) + "\n")
    with open(os.path.join(HERE, "descs.json"), "w") as fh:
        json.dump({k: {"blob": v.blob.hex(), "root": v.root_type} for k, v in flats.items()}, fh)
    codes = {}
    for r in rows:
        codes[r["ret"] & 0xFF] = codes.get(r["ret"] & 0xFF, 0) + 1
    print(len(rows), "rows; status codes:", sorted(codes.items()))


if __name__ == "__main__":
    main()
