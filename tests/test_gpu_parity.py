"""GPU parity: the HIP transcoder (through the C ABI) against the reference-
generated golden vectors and the oracle, bit-exact (integer/byte work: Thrift
bytes and packed status words must be identical)."""
import random
import zlib

import numpy as np
import pytest

import oracle
import fuzz
from dynamicgo_amd import conv, thrift as T, workloads as W

pytestmark = pytest.mark.gpu


def _checker():
    return oracle.RefOracle() or oracle.PortOracle()


NO_FAST = 1 << 17  # DG_F_NO_FAST_PATH: every message on the exact machine
NO_WAVE = 1 << 18  # DG_F_NO_WAVE_PATH: lane kernel (lane fast path + exact machine) only


def _run_rows(rows, flats, extra=0):
    """Group golden rows by (desc, flags) and run each group as one batch."""
    groups = {}
    for i, (name, flags, js, ret, out) in enumerate(rows):
        groups.setdefault((name, flags), []).append(i)
    bad = []
    for (name, flags), idx in groups.items():
        cv = conv.BinaryConv(conv.Options())
        cv.opts = conv.Options()
        msgs = [rows[i][2] for i in idx]
        outs, rets = _raw_batch(flats[name], msgs, flags | extra)
        for k, i in enumerate(idx):
            exp_ret, exp_out = rows[i][3], rows[i][4]
            if int(rets[k]) != exp_ret or outs[k] != exp_out:
                bad.append((name, hex(flags), rows[i][2][:60], hex(int(rets[k])), hex(exp_ret)))
    return bad


def _raw_batch(flat, msgs, flags):
    """dg_j2t_batch_host with an explicit flag word."""
    import ctypes as C
    from dynamicgo_amd import _lib
    ctx = conv.default_context()
    n = len(msgs)
    a, off = W.arena(msgs)
    cap = int(off[-1]) * 16 + 64 * n + 65536
    out = np.zeros(cap, dtype=np.uint8)
    oo = np.zeros(n + 1, dtype=np.uint64)
    rets = np.zeros(n, dtype=np.uint64)
    need = C.c_uint64(0)
    _lib.check(_lib.lib().dg_j2t_batch_host(ctx.h, ctx.desc(flat), flat.root_type, a.ctypes.data, off.ctypes.data,
                                            n, flags, out.ctypes.data, cap, oo.ctypes.data, rets.ctypes.data,
                                            C.byref(need)))
    return [out[int(oo[i]):int(oo[i + 1])].tobytes() for i in range(n)], rets


@pytest.mark.parametrize("extra", [0, NO_WAVE, NO_FAST, "wave-all"],
                         ids=["hybrid", "lane-fast+exact", "exact-only", "wave-all"])
def test_golden_vectors(golden, extra, knob):
    rows, flats = golden
    if extra == "wave-all":
        knob("wave_min", 0)
        extra = 0
    bad = _run_rows(rows, flats, extra)
    assert not bad, bad[:8]


@pytest.mark.parametrize("which", ["D1", "D2", "D3", "simple", "nesting", "example3", "null", "nesting2"])
def test_fuzz_vs_oracle(which):
    from schemas import probe, idl_desc
    td = {"D1": lambda: probe("D1"), "D2": lambda: probe("D2"), "D3": lambda: probe("D3"),
          "simple": lambda: idl_desc("baseline.thrift", "SimpleMethod"),
          "nesting": lambda: idl_desc("baseline.thrift", "NestingMethod"),
          "nesting2": lambda: idl_desc("baseline.thrift", "Nesting2Method"),
          "example3": lambda: idl_desc("example3.thrift", "ExampleMethod"),
          "null": lambda: idl_desc("null.thrift", "NullTest")}[which]()
    fl = T.flatten(td)
    chk = _checker()
    # a fixed seed per schema (str hash() is salted per process); see
    # tests/test_oracle.py::test_unterminated_string_block_tail for the one
    # malformed-input class where the reference's verdict is undefined
    rng = random.Random(zlib.crc32(which.encode()) & 0xffff)
    for flags in (0x1, 0x0, 0x11, 0x5, 0x23, 0x83, 0x41, 0x100, 0x201, NO_FAST | 0x1, NO_FAST | 0x83,
                  NO_WAVE | 0x1, NO_WAVE | 0x83):
        msgs = [fuzz.gen_message(rng, td, mutate_p=rng.random() < 0.5) for _ in range(300)]
        outs, rets = _raw_batch(fl, msgs, flags)
        for m, o, r in zip(msgs, outs, rets):
            er, eo = chk.j2t(fl, m, flags)
            assert (int(r), o) == (er, eo), (which, hex(flags), m)


@pytest.mark.parametrize("cfg", ["c2", "c3", "c3-occ4"])
def test_full_batch_vs_oracle(cfg, knob):
    """The bench workloads at full size (65 536 messages), byte-exact, and all
    of them on the fast path (what bench.py measures). C3 runs on the 5-wave
    instance of the wave kernel (max_len <= 16 KiB), c3-occ4 on the other."""
    if cfg == "c3-occ4":
        knob("wave_occ", 4)
        cfg = "c3"
    td, gen, seed = {"c2": (W.simple_desc, W.gen_flat_batch, 42),
                     "c3": (W.nesting_i64_desc, W.gen_nested_batch, 43)}[cfg]
    fl = T.flatten(td())
    msgs = gen(random.Random(seed), 65536)
    ctx = conv.default_context()
    ctx.stats(reset=True)
    outs, rets = _raw_batch(fl, msgs, 1)
    bails, deeps = ctx.stats(reset=True)
    chk = _checker()
    a, off = W.arena(msgs)
    er, eo = chk.j2t_arena(fl, a, off, 1, nthreads=8)
    assert (np.asarray(rets) == er).all()
    assert outs == eo
    assert (bails, deeps) == (0, 0)


@pytest.mark.parametrize("occ", ["auto", "5"])
def test_large_messages_vs_oracle(occ, knob):
    """C4-shaped messages (too large to stage in LDS: global-source path), on
    the 4-wave instance (max_len > 16 KiB) and forced onto the 5-wave one."""
    if occ != "auto":
        knob("wave_occ", occ)
    fl = T.flatten(W.large_desc())
    rng = random.Random(44)
    msgs = W.gen_large_batch(rng, 24, blob_bytes=6000, n_values=300) + W.gen_large_batch(rng, 8)
    ctx = conv.default_context()
    ctx.stats(reset=True)
    outs, rets = _raw_batch(fl, msgs, 1)
    bails, _ = ctx.stats(reset=True)
    chk = _checker()
    for m, o, r in zip(msgs, outs, rets):
        assert (int(r), o) == chk.j2t(fl, m, 1)
    assert bails == 0


def test_deep_nesting_routes_to_deep_kernel():
    """Depth beyond the fast kernel's stack goes through the 4096-deep kernel;
    beyond MAX_RECURSE the reference's ERR_RECURSE_MAX word comes back."""
    deep = T.list_of(T.builtin("i64"))
    for _ in range(60):
        deep = T.list_of(deep)
    fl = T.flatten(deep)
    chk = _checker()
    msgs = [b"[" * 61 + b"[1,2]" + b"]" * 61, b"[" * 30 + b"]" * 30, b"[" * 70]
    outs, rets = _raw_batch(fl, msgs, 1)
    for m, o, r in zip(msgs, outs, rets):
        assert (int(r), o) == chk.j2t(fl, m, 1)
    d1 = T.flatten(__import__("schemas").probe("D1"))
    msgs = [b'{"Z":' + b"[" * k + b"]" * k + b"}" for k in (10, 63, 64, 65, 200, 4094, 4095, 5000)]
    outs, rets = _raw_batch(d1, msgs, 1)
    for m, o, r in zip(msgs, outs, rets):
        assert (int(r), o) == chk.j2t(d1, m, 1), len(m)


def test_output_overflow_rerun():
    """WriteDefaultField on a wide struct: output >> 4x input -> slot overflow
    -> exact-size rerun on the GPU."""
    fields = [T.FieldDescriptor(i, "f%d" % i, T.builtin("i64"), T.DEFAULT) for i in range(1, 200)]
    td = T.struct_type("Wide", fields)
    fl = T.flatten(td)
    msgs = [b"{}", b'{"f1":1}', b"[]", b"{}" * 3]
    outs, rets = _raw_batch(fl, msgs, 0x3)
    chk = _checker()
    for m, o, r in zip(msgs, outs, rets):
        assert (int(r), o) == chk.j2t(fl, m, 0x3)
    assert len(outs[0]) == 199 * 11 + 1


def test_binaryconv_do_api():
    """BinaryConv.Do surface: bytes out, J2TError with the reference's code."""
    cv = conv.BinaryConv(conv.Options())
    td = W.simple_desc()
    out = cv.do(td, W.c1_simple_json())
    assert len(out) == 114
    with pytest.raises(conv.J2TError) as ei:
        cv.do(td, b'{"ByteField":tru}')
    assert ei.value.code == 1 or ei.value.code == 2
    assert cv.do(td, b"null") is None
    assert cv.do(td, b"") == b"\x00"


def test_device_resident_api_torch():
    import torch
    td = W.simple_desc()
    fl = T.flatten(td)
    msgs = W.gen_flat_batch(random.Random(5), 4096)
    a, off = W.arena(msgs)
    dev = torch.device("cuda:0")
    json = torch.from_numpy(a).to(dev)
    in_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    slots = np.zeros(len(msgs) + 1, dtype=np.int64)
    np.cumsum(np.diff(off).astype(np.int64) * 4 + 64, out=slots[1:])
    out = torch.zeros(int(slots[-1]) + 64, dtype=torch.uint8, device=dev)
    out_off = torch.from_numpy(slots).to(dev)
    out_len = torch.zeros(len(msgs), dtype=torch.int32, device=dev)
    ret = torch.zeros(len(msgs), dtype=torch.int64, device=dev)
    cv = conv.BinaryConv(conv.Options())
    cv.do_device(fl, json, in_off, out, out_off, out_len, ret, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    ol = out_len.cpu().numpy()
    chk = _checker()
    for i, m in enumerate(msgs[:512]):
        er, eo = chk.j2t(fl, m, 1)
        assert int(ret[i]) == er
        assert o[slots[i]:slots[i] + ol[i]].tobytes() == eo


def test_utf8_validation_extension_vs_port_oracle():
    """DG_F_VALIDATE_UTF8 (bit 16, extension): GPU vs the port oracle on
    strings with valid and invalid UTF-8 in values and map keys."""
    rng = random.Random(16)
    pieces = [b"a", b"\xc3\xa9", b"\xe4\xb8\xad", b"\xf0\x9f\x98\x80", b"\xff", b"\xc0\x80", b"\xed\xa0\x80",
              b"\xe4\xb8", b"\\n", b"\\u00e9", b" ", b"0123456789"]

    def s():
        return b'"' + b"".join(rng.choice(pieces) for _ in range(rng.randint(0, 12))) + b'"'
    fl = T.flatten(W.nesting_i64_desc())
    msgs = []
    for _ in range(400):
        msgs.append(b'{"String":' + s() + b',"MapStringString":{' + s() + b":" + s() + b'},"ListString":[' +
                    s() + b"," + s() + b'],"Binary":' + s() + b"}")
    chk = oracle.PortOracle()
    for flags in (0x1 | 1 << 16, 0x1 | 1 << 16 | NO_FAST):
        outs, rets = _raw_batch(fl, msgs, flags)
        for m, o, r in zip(msgs, outs, rets):
            assert (int(r), o) == chk.j2t(fl, m, flags), m


def test_utf8_validation_pinned_to_reference_validator():
    """DG_F_VALIDATE_UTF8 verdicts of the GPU (fast paths and
    the exact machine) against the reference's own validator, utf8_validate
    (native/utf8.c:183-212, oracle/_ref), on 1 500 fuzz bodies as a string
    value and as a STRING map key: rejected exactly when utf8_validate
    returns an offset (ERR_INVAL at that byte), otherwise the reference's
    flag-off bytes."""
    from test_oracle import utf8_fuzz_bodies, UTF8_CASES_BODIES
    ref = oracle.RefOracle()
    if ref is None:
        pytest.skip("oracle/_ref not built")
    bodies = UTF8_CASES_BODIES + utf8_fuzz_bodies(62, 1500)
    fs = T.flatten(W.simple_desc())
    fn = T.flatten(W.nesting_i64_desc())
    cases = [(fs, b'{"StringField":"', b'"}'), (fn, b'{"MapStringString":{"', b'":"v"}}')]
    for fl, pre, post in cases:
        msgs = [pre + b + post for b in bodies]
        want = []
        for b, m in zip(bodies, msgs):
            bad = oracle.ref_utf8_validate(b)
            want.append(ref.j2t(fl, m, 1) if bad < 0 else (((b[bad] << 40) | ((len(pre) + bad) << 8) | 2), b""))
        for flags in (0x1 | 1 << 16, 0x1 | 1 << 16 | NO_FAST):
            outs, rets = _raw_batch(fl, msgs, flags)
            got = [(int(r), o if int(r) == 0 else b"") for r, o in zip(rets, outs)]
            assert got == [(r, o if r == 0 else b"") for r, o in want], flags


def test_pack_device_matches_slots():
    """dg_pack_device: the used prefix of every slot, back to back."""
    import torch
    from dynamicgo_amd import _lib
    td = W.nesting_i64_desc()
    fl = T.flatten(td)
    msgs = W.gen_nested_batch(random.Random(9), 3000) + [b"{]", b"", b"{}"]
    a, off = W.arena(msgs)
    dev = torch.device("cuda:0")
    n = len(msgs)
    slots = np.zeros(n + 1, dtype=np.int64)
    np.cumsum((np.diff(off).astype(np.int64) * 4 + 64 + 7) & ~7, out=slots[1:])
    d_json = torch.from_numpy(a).to(dev)
    d_in = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_out = torch.zeros(int(slots[-1]) + 64, dtype=torch.uint8, device=dev)
    d_oo = torch.from_numpy(slots).to(dev)
    d_ol = torch.zeros(n, dtype=torch.int32, device=dev)
    d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
    ctx = conv.default_context()
    L = _lib.lib()
    st = torch.cuda.current_stream()
    _lib.check(L.dg_j2t_batch_device(ctx.h, ctx.desc(fl), fl.root_type, d_json.data_ptr(), d_in.data_ptr(), n, 1,
                                     d_out.data_ptr(), d_oo.data_ptr(), d_ol.data_ptr(), d_ret.data_ptr(), None,
                                     st.cuda_stream))
    d_doff = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(d_ol, 0, dtype=torch.int64, out=d_doff[1:])
    d_pack = torch.full((int(slots[-1]) + 64,), 0xAB, dtype=torch.uint8, device=dev)
    _lib.check(L.dg_pack_device(ctx.h, d_out.data_ptr(), d_oo.data_ptr(), d_ol.data_ptr(), n, d_pack.data_ptr(),
                                d_doff.data_ptr(), st.cuda_stream))
    torch.cuda.synchronize()
    o, ol, doff = d_out.cpu().numpy(), d_ol.cpu().numpy(), d_doff.cpu().numpy()
    want = b"".join(o[slots[i]:slots[i] + ol[i]].tobytes() for i in range(n))
    got = d_pack.cpu().numpy()
    assert got[:len(want)].tobytes() == want
    assert got[len(want)] == 0xAB  # nothing written past the end
    chk = _checker()
    for i in (0, 1, 2, n - 3, n - 2, n - 1):
        er, eo = chk.j2t(fl, msgs[i], 1)
        assert int(d_ret[i]) == er and got[doff[i]:doff[i + 1]].tobytes() == eo


def _lean_decline_msgs(rng):
    """Small messages (<= 512 B) the small kernel's lean fast path declines on
    purpose: unknown fields with nested values, numeric map keys, unset fields
    under the default/require/optional write flags."""
    simple, nest = [], []
    for _ in range(300):
        o = W.simple_obj(rng)
        k = rng.randint(0, 3)
        if k == 0:  # unknown field holding a nested value, somewhere in the object
            o = o[:-1] + ',"Unknown%d":{"a":[1,"x",{"b":null}],"c":-1.5e3}}' % rng.randint(0, 9)
        elif k == 1:  # drop fields so the write flags have unset fields to fill
            o = '{"I32Field":%d,"StringField":"s"}' % rng.randint(-9, 9)
        elif k == 2:
            o = '{"Unknown":[[],{}],' + o[1:]
        simple.append(o.encode())
        m = ",".join('"%d":"v%d"' % (rng.randint(-2**63, 2**63 - 1), i) for i in range(rng.randint(1, 4)))
        nest.append(('{"I64":%d,"MapI64String":{%s},"MapI32I64":{"%d":7}}'
                     % (rng.randint(-99, 99), m, rng.randint(-2**31, 2**31 - 1))).encode())
    return simple, nest


NO_FLAT = 1 << 21  # DG_F_NO_FLAT_PATH: the small kernel even for flat roots


@pytest.mark.parametrize("route", [0, NO_FLAT])
@pytest.mark.parametrize("flags", [1, 1 | 2, 1 | 32, 1 | 128, 1 | 2 | 32 | 128, 0])
def test_small_kernel_declines_vs_oracle(flags, route):
    """The small kernel leaves unknown-field skips, numeric map keys and
    default writes to the list pass (full fast path, then the exact machine):
    the hybrid route must still be bit-exact with the oracle on them (route 0:
    Simple takes the flat kernel, NO_FLAT: the small kernel)."""
    simple, nest = _lean_decline_msgs(random.Random(7 + flags))
    chk = _checker()
    for fl, msgs in ((T.flatten(W.simple_desc()), simple), (T.flatten(W.nesting_desc()), nest)):
        assert max(len(m) for m in msgs) <= 512
        outs, rets = _raw_batch(fl, msgs, flags | route)
        for m, o, r in zip(msgs, outs, rets):
            assert (int(r), o) == chk.j2t(fl, m, flags), m[:200]


@pytest.mark.parametrize("route", [0, NO_FLAT])
def test_small_kernel_wave_staging_vs_oracle(route):
    """Blocks whose JSON span does not fit the stage (large messages between
    small ones) stage per wave; waves whose small messages still do not fit
    read global memory. Both must be bit-exact with the oracle. (Route 0: the
    flat kernel stages per message and lists 257-512 B messages for the wave
    kernel.)"""
    rng = random.Random(11)
    fl = T.flatten(W.simple_desc())
    msgs = []
    for blk in range(12):
        for k in range(256):
            r = rng.random()
            if blk % 3 == 0 and r < 0.05:  # large: the wave kernel's
                msgs.append(('{"StringField":"%s","I32Field":%d}' % ("x" * rng.randint(600, 3000), k)).encode())
            elif blk % 3 == 1 and r < 0.5:  # 400-512 B: the wave's quarter overflows -> global source
                msgs.append(('{"StringField":"%s","ByteField":1}' % ("y" * rng.randint(380, 480))).encode())
            else:
                msgs.append(W.simple_obj(rng).encode())
    chk = _checker()
    outs, rets = _raw_batch(fl, msgs, 1 | route)
    for m, o, r in zip(msgs, outs, rets):
        assert (int(r), o) == chk.j2t(fl, m, 1), m[:120]


@pytest.mark.parametrize("cfg", ["c2x", "c2s"])
def test_reference_options_and_shuffled_keys_vs_oracle(cfg):
    """c2x: the reference benchmark's options (WriteDefaultField +
    EnableValueMapping, flags 0x7, testdata/test/baseline_j2t_test.go:721-737)
    on the C2 batch, where I64Field carries api.js_conv: every message must
    stay on the fast path (inline js_conv, native/thrift.c:514-634).
    c2s: C2 with shuffled key order (the divergence stress). Both at full
    size, byte-exact vs the oracle, zero messages on the exact machine."""
    if cfg == "c2x":
        msgs, flags = W.gen_flat_batch(random.Random(42), 65536), 0x7
    else:
        msgs, flags = W.gen_flat_batch_shuffled(random.Random(42), 65536), 0x1
    fl = T.flatten(W.simple_desc())
    ctx = conv.default_context()
    ctx.stats(reset=True)
    outs, rets = _raw_batch(fl, msgs, flags)
    bails, deeps = ctx.stats(reset=True)
    a, off = W.arena(msgs)
    er, eo = _checker().j2t_arena(fl, a, off, flags, nthreads=8)
    assert (np.asarray(rets) == er).all()
    assert outs == eo
    assert (bails, deeps) == (0, 0)


def test_jsconv_value_forms_vs_oracle():
    """api.js_conv under F_ENABLE_VM on every Thrift type the inline mapping
    supports: quoted and bare numbers, "" (default / empty), strings,
    quoted garbage, the i16 fall-through, and non-js_conv neighbours."""
    rng = random.Random(101)
    F = T.FieldDescriptor
    fields = [F(1, "I8", T.builtin("byte"), vm=T.VM_JSCONV), F(2, "I16", T.builtin("i16"), vm=T.VM_JSCONV),
              F(3, "I32", T.builtin("i32"), vm=T.VM_JSCONV), F(4, "I64", T.builtin("i64"), vm=T.VM_JSCONV),
              F(5, "D", T.builtin("double"), vm=T.VM_JSCONV), F(6, "S", T.builtin("string"), vm=T.VM_JSCONV),
              F(7, "B", T.builtin("bool"), vm=T.VM_JSCONV), F(8, "P", T.builtin("i64")),
              F(9, "Q", T.builtin("i32"), vm=T.VM_JSCONV, default_value=b"\x00\x00\x00\x07")]
    fl = T.flatten(T.struct_type("VM", fields))
    vals = ['"12"', "12", '"-7"', "-7", '""', '"1.5e3"', "1.5e3", '"x"', '"12x"', "null", "true", '"abc"',
            "300", '"70000"', "9223372036854775807", '"9223372036854775808"', "-0", '"-"', "1e400"]
    msgs = []
    for _ in range(3000):
        ks = rng.sample(["I8", "I16", "I32", "I64", "D", "S", "B", "P", "Q"], rng.randint(1, 5))
        msgs.append(("{" + ",".join('"%s":%s' % (k, rng.choice(vals)) for k in ks) + "}").encode())
    chk = _checker()
    for flags in (0x5, 0x7, 0x1, 0x27):
        outs, rets = _raw_batch(fl, msgs, flags)
        for m, o, r in zip(msgs, outs, rets):
            assert (int(r), o) == chk.j2t(fl, m, flags), (hex(flags), m)
