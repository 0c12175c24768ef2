"""GPU parity of the reverse path (Thrift binary -> JSON, conv/t2j): the HIP
kernels through the C ABI against the t2j checker (oracle/ref_harness.c
dgref_t2j: the reference's control flow over the reference's own native
quote / i64toa / f64toa / b64encode), byte for byte and status word for
status word; plus the reference's own known answers (conv/t2j/conv_test.go
TestInt2String)."""
import ctypes as C
import math
import random
import struct

import numpy as np
import pytest

import oracle
import t2jgen
from dynamicgo_amd import _lib, conv, t2j, thrift as T, workloads as W

pytestmark = pytest.mark.gpu

B8, I64S, NULLNAN, NOB64, DISALLOW, WDEF, WREQ, WOPT, VM = (1 << k for k in range(9))
OPTS = [0, B8 | I64S, NULLNAN, NOB64, DISALLOW, WDEF | WREQ | WOPT, VM, B8 | I64S | NULLNAN | NOB64 | WDEF | WOPT | VM]


@pytest.fixture(scope="module")
def chk():
    o = oracle.RefT2JOracle()
    if o is None:
        pytest.skip("oracle/_ref not built")
    return o


def gpu_t2j(flat, msgs, opts, root=None):
    """dg_t2j_batch_host over the messages -> (outs, rets)."""
    ctx = conv.default_context()
    n = len(msgs)
    a, off = W.arena(msgs)
    cap = int(off[-1]) * 8 + 64 * n + 65536
    out = np.zeros(cap, dtype=np.uint8)
    oo = np.zeros(n + 1, dtype=np.uint64)
    rets = np.zeros(max(n, 1), dtype=np.uint64)
    need = C.c_uint64(0)
    _lib.check(_lib.lib().dg_t2j_batch_host(ctx.h, ctx.desc_t2j(flat), flat.root_type if root is None else root,
                                            a.ctypes.data, off.ctypes.data, n, opts, out.ctypes.data, cap,
                                            oo.ctypes.data, rets.ctypes.data, C.byref(need)))
    return [out[int(oo[i]):int(oo[i + 1])].tobytes() for i in range(n)], rets[:n]


def compare(chk, flat, msgs, opts, root=None):
    side = T.flatten_t2j(flat)
    outs, rets = gpu_t2j(flat, msgs, opts, root)
    bad = []
    for i, m in enumerate(msgs):
        er, eo = chk.t2j(flat, side, m, opts, root)
        if int(rets[i]) != er or outs[i] != eo:
            bad.append((i, hex(int(rets[i])), hex(er), outs[i][:80], eo[:80], m[:40].hex()))
    return bad


def test_int2string_known_answers():
    """conv/t2j/conv_test.go:332-386 through the Python mirror."""
    from schemas import idl_desc
    from test_t2j_oracle import int2float_thrift
    td = idl_desc("example3.thrift", "Int2FloatMethod")
    src = int2float_thrift()
    cv = t2j.BinaryConv(conv.Options(EnableValueMapping=True))
    assert cv.do(td, src) == '{"Int32":"1","Float64":"3.14","中文":"hello","Int64":2,"Subfix":0.92653}'.encode()
    cv = t2j.BinaryConv(conv.Options())
    assert cv.do(td, src) == '{"Int32":1,"Float64":3.14,"中文":"hello","Int64":2,"Subfix":0.92653}'.encode()
    cv = t2j.BinaryConv(conv.Options(Int642String=True))
    assert cv.do(td, src) == '{"Int32":1,"Float64":3.14,"中文":"hello","Int64":"2","Subfix":0.92653}'.encode()
    with pytest.raises(t2j.T2JError) as ei:
        t2j.BinaryConv(conv.Options()).do(td, int2float_thrift(math.nan))
    assert ei.value.behavior == "ErrWrite"
    cv = t2j.BinaryConv(conv.Options(EncodeNullJSONForInfOrNan=True))
    assert cv.do(td, int2float_thrift(math.inf)) == \
        '{"Int32":1,"Float64":3.14,"中文":"hello","Int64":2,"Subfix":null}'.encode()


@pytest.mark.parametrize("opts", OPTS)
def test_random_parity(chk, opts):
    td = t2jgen.all_types_desc()
    fl = T.flatten(td)
    rng = random.Random(1000 + opts)
    msgs = [t2jgen.gen_thrift(rng, td) for _ in range(1500)]
    msgs += [t2jgen.mutate(rng, t2jgen.gen_thrift(rng, td)) for _ in range(700)]
    bad = compare(chk, fl, msgs, opts)
    assert not bad, bad[:5]


@pytest.mark.parametrize("wmin", ["512", "1", "0"])
def test_numbers_and_strings_exhaustive(chk, wmin, knob):
    """Many doubles (every f64toa format branch), integers and strings, on the
    wave kernel (t2j_wave.h: long messages by default, every message with
    t2j_wave_min 1) and on the lane kernel alone (0)."""
    knob("t2j_wave_min", wmin)
    td = T.struct_type("N", [T.FieldDescriptor(1, "d", T.list_of(T.builtin("double")), T.OPTIONAL),
                             T.FieldDescriptor(2, "i", T.list_of(T.builtin("i64")), T.OPTIONAL),
                             T.FieldDescriptor(3, "s", T.list_of(T.builtin("string")), T.OPTIONAL),
                             T.FieldDescriptor(4, "b", T.list_of(T.builtin("binary")), T.OPTIONAL)])
    fl = T.flatten(td)
    rng = random.Random(5)
    msgs = []
    for _ in range(400):
        ds = [t2jgen.rdouble(rng) for _ in range(40)]
        ds += [float(10 ** k) for k in range(-8, 23)] + [1.5 * 10 ** k for k in range(-8, 23)]
        iv = [t2jgen.rint(rng, 64) for _ in range(20)] + [-(1 << 63), (1 << 63) - 1, 10 ** 8, 10 ** 16 - 1]
        ss = [t2jgen.rbytes(rng, 40) for _ in range(10)] + [bytes(range(256)), b""]
        bs = [bytes(rng.randrange(256) for _ in range(rng.randrange(20))) for _ in range(10)]
        m = b"\x0f\x00\x01\x04" + struct.pack(">i", len(ds)) + b"".join(struct.pack(">d", d) for d in ds)
        m += b"\x0f\x00\x02\x0a" + struct.pack(">i", len(iv)) + b"".join(struct.pack(">q", v) for v in iv)
        m += b"\x0f\x00\x03\x0b" + struct.pack(">i", len(ss)) + b"".join(struct.pack(">i", len(s)) + s for s in ss)
        m += b"\x0f\x00\x04\x0b" + struct.pack(">i", len(bs)) + b"".join(struct.pack(">i", len(s)) + s for s in bs)
        msgs.append(m + b"\x00")
    for opts in (0, NOB64):
        bad = compare(chk, fl, msgs, opts)
        assert not bad, bad[:3]


@pytest.mark.parametrize("depth", [1, 11, 12, 13, 40, 1000, 4095])
def test_deep_chain(chk, depth):
    """Nesting beyond the LDS frames reruns on the deep pass, same bytes."""
    fl = T.flatten(t2jgen.chain_desc())
    msgs = [t2jgen.chain_thrift(depth), t2jgen.chain_thrift(2)] * 3
    assert not compare(chk, fl, msgs, 0)


def test_deeper_than_frames():
    """Past 4096 containers the GPU reports DG_T2J_E_DEPTH (Go recurses on)."""
    fl = T.flatten(t2jgen.chain_desc())
    outs, rets = gpu_t2j(fl, [t2jgen.chain_thrift(5000), t2jgen.chain_thrift(3)], 0)
    assert int(rets[0]) & 0xFF == 8 and outs[0] == b""
    assert int(rets[1]) == 0 and outs[1] == b'{"next":{"next":{"v":7}}}'


@pytest.mark.parametrize("levels", [5, 20, 1021, 1022, 1023, 1100])
def test_skip_depth_limit(chk, levels):
    """An unknown field of nested lists: skipType's MaxSkipDepth (1023,
    thrift/binary_skip.go:24) holds on the GPU too."""
    td = T.struct_type("S", [T.FieldDescriptor(1, "a", T.builtin("i32"), T.OPTIONAL)])
    fl = T.flatten(td)
    body = b"\x0f" + struct.pack(">i", 1)
    inner = b"\x08" + struct.pack(">i", 1) + struct.pack(">i", 9)
    v = body * (levels - 1) + inner
    m = b"\x0f\x00\x63" + v + b"\x08\x00\x01" + struct.pack(">i", 3) + b"\x00"
    # unknown struct-of-structs as well
    s = b"\x0c\x00\x64" + b"\x0c\x00\x01" * (levels - 1) + b"\x00" * levels + b"\x00"
    assert not compare(chk, fl, [m, s, m[:len(m) // 2]], 0)


def test_wide_structs_vs_checker(chk):
    """Structs of more than 64 fields (multi-word requires bitmaps,
    HandleRequires over every word, conv/t2j/impl.go:268-290): rerun by the
    deep pass with per-lane requires words, nested inside lists and inside
    each other, every requireness, byte-exact against the checker."""
    rng = random.Random(21)
    for n in (65, 70, 150):
        fs = [T.FieldDescriptor(i + 1, f"f{i}", T.builtin("i32"), (T.OPTIONAL, T.DEFAULT, T.REQUIRED)[i % 3])
              for i in range(n)]
        wide = T.struct_type("Wide%d" % n, fs)
        outer = T.struct_type("Outer", [T.FieldDescriptor(1, "w", wide, T.OPTIONAL),
                                        T.FieldDescriptor(2, "ws", T.list_of(wide), T.OPTIONAL),
                                        T.FieldDescriptor(3, "x", T.builtin("i64"), T.OPTIONAL)])
        fl = T.flatten(outer)

        def one():
            ids = rng.sample(range(1, n + 1), rng.randint(0, n))
            if rng.random() < 0.5:
                ids = sorted(set(ids) | {i for i in range(3, n + 1, 3)})  # every REQUIRED field
            return b"".join(b"\x08" + struct.pack(">hi", i, rng.randint(-9, 9)) for i in ids) + b"\x00"
        msgs = []
        for _ in range(60):
            k = rng.randint(0, 3)
            m = b"\x0c\x00\x01" + one() + b"\x0f\x00\x02\x0c" + struct.pack(">i", k) + b"".join(one() for _ in range(k))
            msgs.append(m + b"\x0a\x00\x03" + struct.pack(">q", 5) + b"\x00")
        for opts in (0, WREQ, WDEF | WREQ | WOPT):
            assert not compare(chk, fl, msgs, opts), (n, opts)
        outs, rets = gpu_t2j(fl, msgs, WREQ)
        assert all(int(r) == 0 for r in rets)


def test_defaults_vs_checker(chk):
    """An unset field with an IDL default is written as DefaultValue().
    JSONValue() (scalar and string constants from their Thrift bytes; a
    container constant stays NEEDS_HOST, on both sides)."""
    td = t2jgen.all_types_desc(with_default=True)
    fl = T.flatten(td)
    rng = random.Random(9)
    msgs = [t2jgen.gen_thrift(rng, td) for _ in range(200)]
    for opts in (0, WOPT, WDEF | WREQ | WOPT):
        assert not compare(chk, fl, msgs, opts)
    outs, rets = gpu_t2j(fl, msgs, WDEF | WREQ | WOPT)
    assert sum(int(r) == 0 for r in rets) > 100


def test_scalar_and_container_roots(chk):
    """Non-struct root descriptors (doRecurse on the root type directly)."""
    rng = random.Random(3)
    cases = [(T.builtin("i64"), [struct.pack(">q", -5), b"\x01"]),
             (T.builtin("string"), [struct.pack(">i", 3) + b'a"b', struct.pack(">i", 9) + b"ab"]),
             (T.builtin("double"), [struct.pack(">d", 0.1), struct.pack(">d", math.nan)]),
             (T.list_of(T.builtin("i32")), [b"\x08" + struct.pack(">i", 2) + struct.pack(">ii", 1, -2),
                                             b"\x0b" + struct.pack(">i", 0)]),
             (T.map_of(T.builtin("string"), T.builtin("i32")),
              [b"\x0b\x08" + struct.pack(">i", 1) + struct.pack(">i", 1) + b"k" + struct.pack(">i", 4)]),
             (T.map_of(T.builtin("bool"), T.builtin("i32")), [b"\x02\x08" + struct.pack(">i", 1) + b"\x01" +
                                                                struct.pack(">i", 4)])]
    for td, msgs in cases:
        fl = T.flatten(td)
        msgs = msgs + [t2jgen.mutate(rng, m) for m in msgs] + [b""]
        assert not compare(chk, fl, msgs, 0)


def test_empty_and_truncated(chk):
    td = t2jgen.all_types_desc()
    fl = T.flatten(td)
    rng = random.Random(11)
    m = t2jgen.gen_thrift(rng, td)
    msgs = [b"", b"\x00"] + [m[:k] for k in range(0, len(m), max(1, len(m) // 60))]
    assert not compare(chk, fl, msgs, 0)


def test_overflow_rerun(chk):
    """JSON much larger than dg_t2j_slot_bound (control bytes -> \\u00xx):
    the host entry point reruns those messages with exact slots."""
    td = T.struct_type("S", [T.FieldDescriptor(1, "s", T.builtin("string"), T.OPTIONAL)])
    fl = T.flatten(td)
    msgs = []
    for k in (0, 1, 7, 100, 5000):
        s = b"\x01" * k
        msgs.append(b"\x0b\x00\x01" + struct.pack(">i", k) + s + b"\x00")
    assert not compare(chk, fl, msgs, 0)


def test_roundtrip_c2(chk):
    """C2's JSON through the GPU j2t, then the Thrift bytes back through the
    GPU t2j: identical to the checker, and JSON-equivalent to the input
    (t2j(j2t(x)) keeps every value)."""
    import json
    rng = random.Random(21)
    td = W.simple_desc()
    fl = T.flatten(td)
    js = W.gen_flat_batch(rng, 500)
    cv = conv.BinaryConv(conv.Options())
    thr, rets = cv.do_batch(td, js)
    assert not any(int(r) for r in rets)
    bad = compare(chk, fl, thr, 0)
    assert not bad, bad[:3]
    outs, _ = gpu_t2j(fl, thr, 0)
    for a, b in zip(js, outs):
        ja, jb = json.loads(a), json.loads(b)
        assert set(ja) <= set(jb)


def test_device_entry_point(chk):
    """dg_t2j_batch_device over torch tensors on the current stream:
    overflowing slots report DG_ST_OUT_OVERFLOW with the bytes needed."""
    import torch
    td = t2jgen.all_types_desc()
    fl = T.flatten(td)
    side = T.flatten_t2j(fl)
    rng = random.Random(13)
    msgs = [t2jgen.gen_thrift(rng, td) for _ in range(3000)]
    a, off = W.arena(msgs)
    n = len(msgs)
    lens = np.diff(off).astype(np.int64)
    slots = ((lens // 2 + 8 + 7) // 8) * 8  # small on purpose: most overflow
    oo = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(slots, out=oo[1:])
    dev = torch.device("cuda:0")
    d_src = torch.from_numpy(a).to(dev)
    d_in = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_oo = torch.from_numpy(oo).to(dev)
    d_out = torch.zeros(int(oo[-1]) + 64, dtype=torch.uint8, device=dev)
    d_ol = torch.zeros(n, dtype=torch.int32, device=dev)
    d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
    t2j.BinaryConv(conv.Options()).do_device(td, d_src, d_in, d_out, d_oo, d_ol, d_ret)
    torch.cuda.synchronize()
    out, ol, ret = d_out.cpu().numpy(), d_ol.cpu().numpy(), d_ret.cpu().numpy().view(np.uint64)
    over = 0
    for i, m in enumerate(msgs):
        er, eo = chk.t2j(fl, side, m, 0)
        if int(ret[i]) & 0xFF == 0xF0:
            over += 1
            assert er == 0 and int(ol[i]) == len(eo)
            continue
        assert int(ret[i]) == er
        if er == 0:
            assert out[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() == eo
    assert over > 0


@pytest.mark.parametrize("spread", ["1", "2", "4", "auto"])
def test_spreads_vs_checker(chk, spread, knob):
    """The LDS-frame pass at each lanes-per-message spread (t2j_kern.hip), and
    the host's own choice from the longest message: random all-types
    messages (with mutations) and nested C3 Thrift, byte-exact."""
    knob("t2j_wave_min", 0)  # the lane pass for every message
    if spread != "auto":
        knob("t2j_spread", spread)
    td = t2jgen.all_types_desc()
    fl = T.flatten(td)
    rng = random.Random(77)
    msgs = [t2jgen.gen_thrift(rng, td) for _ in range(700)]
    msgs += [t2jgen.mutate(rng, t2jgen.gen_thrift(rng, td)) for _ in range(300)]
    bad = compare(chk, fl, msgs, 0)
    assert not bad, bad[:5]
    ntd = W.nesting_i64_desc()
    nfl = T.flatten(ntd)
    thr, rets = conv.BinaryConv(conv.Options()).do_batch(ntd, W.gen_nested_batch(random.Random(43), 300))
    assert not any(int(r) for r in rets)
    bad = compare(chk, nfl, thr, 0)
    assert not bad, bad[:3]


def test_device_entry_point_ml(chk):
    """dg_t2j_batch_device_ml (the longest message given) on C3-sized Thrift:
    byte-exact through the spread-4 instance."""
    import torch
    ntd = W.nesting_i64_desc()
    fl = T.flatten(ntd)
    side = T.flatten_t2j(fl)
    thr, rets = conv.BinaryConv(conv.Options()).do_batch(ntd, W.gen_nested_batch(random.Random(44), 2000))
    assert not any(int(r) for r in rets)
    a, off = W.arena(thr)
    n = len(thr)
    lens = np.diff(off).astype(np.int64)
    oo = np.zeros(n + 1, dtype=np.int64)
    np.cumsum((lens * 3 + 64 + 7) // 8 * 8, out=oo[1:])
    dev = torch.device("cuda:0")
    ctx = conv.default_context()
    dh = ctx.desc_t2j(fl)
    d_src = torch.from_numpy(a).to(dev)
    d_in = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_oo = torch.from_numpy(oo).to(dev)
    d_out = torch.zeros(int(oo[-1]) + 64, dtype=torch.uint8, device=dev)
    d_ol = torch.zeros(n, dtype=torch.int32, device=dev)
    d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
    _lib.check(_lib.lib().dg_t2j_batch_device_ml(ctx.h, dh, fl.root_type, d_src.data_ptr(), d_in.data_ptr(), n, 0,
                                                 d_out.data_ptr(), d_oo.data_ptr(), d_ol.data_ptr(),
                                                 d_ret.data_ptr(), torch.cuda.current_stream().cuda_stream,
                                                 int(lens.max())))
    torch.cuda.synchronize()
    out, ol, ret = d_out.cpu().numpy(), d_ol.cpu().numpy(), d_ret.cpu().numpy()
    for i, m in enumerate(thr):
        er, eo = chk.t2j(fl, side, m, 0)
        assert (int(ret[i]), out[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes()) == (er, eo)


def _example3(kind):
    import os
    idl = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "idl", "example3.thrift")
    fn = T.new_descriptor_from_path(idl).functions()["ExampleMethod"]
    return (fn.response() if kind == "resp" else fn.request()).struct.fields[0].type


@pytest.mark.parametrize("kind", ["resp", "req"])
def test_reference_fixtures_example3(kind):
    """conv/t2j/conv_test.go:138-155 (TestConvThrift2JSON): the reference's
    own testdata/data/example3{resp,req}.bin converted on the GPU equal
    example3{resp,req}.json semantically (the Go test compares the decoded
    structs), and the round trip JSON -> Thrift (j2t, GPU) -> JSON (t2j, GPU)
    keeps every value. Fixtures copied verbatim into tests/golden/."""
    import json
    import os
    g = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    td = _example3(kind)
    tb = open(os.path.join(g, "example3%s.bin" % kind), "rb").read()
    js = open(os.path.join(g, "example3%s.json" % kind), "rb").read()
    out = t2j.BinaryConv(conv.Options()).do(td, tb)
    assert json.loads(out) == json.loads(js)
    thrift = conv.BinaryConv(conv.Options()).do(td, js)
    assert len(thrift) == len(tb)
    assert json.loads(t2j.BinaryConv(conv.Options()).do(td, thrift)) == json.loads(js)


def test_error_behaviors_match_impl_go(chk):
    """conv/t2j/impl.go wraps a truncated BYTE/I16/I32/I64/DOUBLE read as
    meta.ErrWrite (:200-236), a BOOL/STRING one as ErrRead, and any map-key
    failure as ErrConvert (:355-358); the GPU status words carry those
    classes (E_WRITE 9 / E_CONVERT 10) and match the checker."""
    i32 = T.struct_type("S", [(1, "a", T.builtin("i32")), (2, "s", T.builtin("string")),
                              (3, "m", T.map_of(T.builtin("i64"), T.builtin("string"))),
                              (4, "b", T.map_of(T.builtin("bool"), T.builtin("string")))])
    fl = T.flatten(i32)
    msgs = [bytes([8, 0, 1, 0, 0]),                                   # i32 cut after 2 bytes
            bytes([11, 0, 2, 0, 0, 0, 5]) + b"ab",                    # string cut
            bytes([13, 0, 3, 10, 11, 0, 0, 0, 1, 0, 0, 0]),           # i64 map key cut
            bytes([13, 0, 4, 2, 11, 0, 0, 0, 1, 1, 0, 0, 0, 0, 0])]   # bool map key: unsupported
    outs, rets = gpu_t2j(fl, msgs, 0)
    side = T.flatten_t2j(fl)
    for m, r in zip(msgs, rets):
        assert chk.t2j(fl, side, m, 0)[0] == int(r)
    beh = [t2j.T2JError(int(r)).behavior for r in rets]
    assert beh == ["ErrWrite", "ErrRead", "ErrConvert", "ErrConvert"], beh


@pytest.mark.parametrize("opts", OPTS)
def test_wave_path_random_parity(chk, opts, knob):
    """Every message through the wave kernel (t2j_wave_min 1): random
    all-types messages, mutated ones (truncations, bad types: the wave kernel
    bails them to the lane kernel), under every option set."""
    knob("t2j_wave_min", 1)
    td = t2jgen.all_types_desc()
    fl = T.flatten(td)
    rng = random.Random(2000 + opts)
    msgs = [t2jgen.gen_thrift(rng, td) for _ in range(1200)]
    msgs += [t2jgen.mutate(rng, t2jgen.gen_thrift(rng, td)) for _ in range(600)]
    bad = compare(chk, fl, msgs, opts)
    assert not bad, bad[:5]


def test_wave_path_nested_and_escapes(chk, knob):
    """C3-shaped Thrift (lists of structs, maps with i64 / string keys)
    through the wave kernel, with map keys and values that need escapes at
    every 8-byte phase, long strings (copy tasks) and long binaries (base64
    tasks)."""
    knob("t2j_wave_min", 64)
    ntd = W.nesting_i64_desc()
    nfl = T.flatten(ntd)
    rng = random.Random(44)
    js = W.gen_nested_batch(rng, 400)
    thr, rets = conv.BinaryConv(conv.Options()).do_batch(ntd, js)
    assert not any(int(r) for r in rets)
    bad = compare(chk, nfl, thr, 0)
    assert not bad, bad[:3]
    td = T.struct_type("E", [
        T.FieldDescriptor(1, "m", T.map_of(T.builtin("string"), T.builtin("string")), T.OPTIONAL),
        T.FieldDescriptor(2, "b", T.builtin("binary"), T.OPTIONAL),
        T.FieldDescriptor(3, "s", T.builtin("string"), T.OPTIONAL)])
    fl = T.flatten(td)
    msgs = []
    for k in range(300):
        kv = []
        for j in range(rng.randrange(1, 6)):
            key = bytes(rng.choice(b'ab"\\\n\t\x01\x1fz') for _ in range(rng.randrange(0, 30)))
            val = bytes(rng.choice(b'xy"\\\r\x02q') for _ in range(rng.randrange(0, 70)))
            kv.append(struct.pack(">i", len(key)) + key + struct.pack(">i", len(val)) + val)
        m = b"\x0d\x00\x01\x0b\x0b" + struct.pack(">i", len(kv)) + b"".join(kv)
        blob = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 200)))
        m += b"\x0b\x00\x02" + struct.pack(">i", len(blob)) + blob
        txt = bytes(rng.choice(b"abcdefgh") for _ in range(rng.randrange(0, 300)))
        m += b"\x0b\x00\x03" + struct.pack(">i", len(txt)) + txt + b"\x00"
        msgs.append(m)
    for opts in (0, NOB64):
        bad = compare(chk, fl, msgs, opts)
        assert not bad, bad[:3]


@pytest.mark.parametrize("wmin", [64, 256])
def test_wave_path_overlapped(chk, knob, wmin):
    """t2j_overlap 1: the route kernel lists the long messages, the wave
    kernel (and its bails' list pass) runs on the scratch's second stream
    beside the lane pass, which skips them. Mixed short / long / mutated
    messages, so all three passes and the deep pass have work."""
    knob("t2j_overlap", 1)
    knob("t2j_wave_min", wmin)
    ntd = W.nesting_i64_desc()
    nfl = T.flatten(ntd)
    rng = random.Random(45 + wmin)
    js = W.gen_nested_batch(rng, 500)
    thr, rets = conv.BinaryConv(conv.Options()).do_batch(ntd, js)
    assert not any(int(r) for r in rets)
    thr = list(thr) + [t2jgen.mutate(rng, bytes(m)) for m in thr[:150]]
    bad = compare(chk, nfl, thr, 0)
    assert not bad, bad[:3]


# ---- the Go-side options: ConvertException, EnableThriftBase, agw.body_dynamic ----
CONV_EXC, SKIP_BASE = 1 << 9, 1 << 10


def test_agw_body_dynamic_read(chk):
    """TestAGWBodyDynamic (conv/t2j/conv_test.go:266-286) through Do, and a
    fuzz of the body_dynamic read against the checker."""
    from test_t2j_oracle import _example3_svc, error_resp_thrift
    td = _example3_svc().functions()["ErrorMethod"].response().struct.fields[0].type
    assert t2j.BinaryConv(conv.Options(EnableValueMapping=True)).do(td, error_resp_thrift()) == \
        b'{"Int64":1,"Xjson":{"b":1}}'
    assert t2j.BinaryConv(conv.Options()).do(td, error_resp_thrift()) == b'{"Int64":1,"Xjson":"{\\"b\\":1}"}'
    fl = T.flatten(td)
    rng = random.Random(4)
    msgs = []
    for k in range(500):
        body = bytes(rng.choice(b'{}[]":,ab01 ') for _ in range(rng.randint(0, 40)))
        m = b"\x0a\x00\x02" + struct.pack(">q", k) + b"\x0b\x00\x04" + struct.pack(">i", len(body)) + body + b"\x00"
        if k % 7 == 0:
            m = m[:rng.randint(0, len(m))]  # truncated
        msgs.append(m)
    for opts in (VM, 0, VM | WDEF):
        assert not compare(chk, fl, msgs, opts)


def test_convert_exception(chk):
    """TestException (conv/t2j/conv_test.go:310-330): Do raises with the
    exception's JSON as the text; the device keeps the JSON (status 11)."""
    from test_t2j_oracle import _example3_svc, exception_result_thrift
    td = _example3_svc().functions()["ExampleMethod"].response()
    with pytest.raises(t2j.T2JException) as ei:
        t2j.BinaryConv(conv.Options(ConvertException=True)).do(td, exception_result_thrift())
    assert str(ei.value) == '{"code":400,"msg":"this is an exception"}'
    fl = T.flatten(td)
    succ_only = exception_result_thrift()
    succ_only = succ_only[:succ_only.index(b"\x0c\x00\x01")] + b"\x00"
    msgs = [exception_result_thrift(), succ_only, exception_result_thrift()[:-3]]
    for opts in (CONV_EXC, CONV_EXC | WDEF | WREQ | WOPT, 0):
        assert not compare(chk, fl, msgs, opts)


def test_response_base(chk):
    """TestThriftResponseBase (conv/t2j/conv_test.go:232-264): with a
    context BaseResp the JSON has no BaseResp and the context object holds
    what it held."""
    import json
    import os
    from test_t2j_oracle import _example3_svc
    td = _example3_svc(T.Options(enable_thrift_base=True)).functions()["ExampleMethod"].response().struct.fields[0].type
    src = open(os.path.join(os.path.dirname(__file__), "golden", "example3resp.bin"), "rb").read()
    cv = t2j.BinaryConv(conv.Options(EnableThriftBase=True))
    plain = json.loads(cv.do(td, src))
    base = t2j.BaseResp()
    got = json.loads(cv.do(td, src, base=base))
    want = plain.pop("BaseResp")
    assert got == plain
    assert (base.StatusMessage, base.StatusCode, base.Extra or {}) == \
        (want["StatusMessage"], want["StatusCode"], want.get("Extra") or {})
    fl = T.flatten(td)
    side = T.flatten_t2j(fl)
    outs, errs = cv.do_batch_errors(td, [src] * 3, bases=[t2j.BaseResp() for _ in range(3)])
    assert all(e is None for e in errs)
    r, js, aux = chk.t2j2(fl, side, src, SKIP_BASE)
    assert outs[0] == js
    # a mixed batch: only the messages whose context holds a BaseResp skip
    # the field (readResponseBase returns false without one, impl.go:54-58)
    bases = [t2j.BaseResp(), None, t2j.BaseResp(), None]
    outs, errs = cv.do_batch_errors(td, [src] * 4, bases=bases)
    assert all(e is None for e in errs)
    for k in range(4):
        alone = cv.do(td, src, base=t2j.BaseResp() if bases[k] is not None else None)
        assert outs[k] == alone, k
    assert json.loads(outs[1]) == dict(plain, BaseResp=want)
    assert json.loads(outs[0]) == plain


# ---- EnableHttpMapping: the device's writeHttpValue stops against the harness ----
HM = 1 << 11


def gpu_t2j_ans(flat, msgs, opts, answers):
    """dg_t2j_batch_host_cb with each message's answers -> (outs, rets)."""
    ctx = conv.default_context()
    n = len(msgs)
    a, off = W.arena(msgs)
    cap = int(off[-1]) * 8 + 64 * n + 65536
    out = np.zeros(cap, dtype=np.uint8)
    oo = np.zeros(n + 1, dtype=np.uint64)
    rets = np.zeros(max(n, 1), dtype=np.uint64)
    need = C.c_uint64(0)
    tab = (_lib.VMEntry * max(n, 1))()
    blob = bytearray()
    for k, an in enumerate(answers):
        tab[k].off, tab[k].count = len(blob), len(an)
        blob += an
    ab = np.frombuffer(bytes(blob) + b"\0" * 8, dtype=np.uint8)
    cb = _lib.CBTables(None, 0, C.cast(tab, C.c_void_p), ab.ctypes.data, len(blob))
    _lib.check(_lib.lib().dg_t2j_batch_host_cb(ctx.h, ctx.desc_t2j(flat), flat.root_type, a.ctypes.data,
                                               off.ctypes.data, n, opts, out.ctypes.data, cap, oo.ctypes.data,
                                               rets.ctypes.data, C.byref(need), None, C.byref(cb)))
    return [out[int(oo[i]):int(oo[i + 1])].tobytes() for i in range(n)], rets[:n]


def hm_desc():
    """Mapped fields at the root, in a root field's struct (resp passed on),
    in list / map elements (nil resp), inside a mapped container (its JSON
    conversion passes resp), with required / optional / default ones."""
    hdr = lambda k: [("api.header", k)]
    s2 = T.struct_type("S2", [T.FieldDescriptor(1, "v", T.builtin("i32"), T.OPTIONAL, http_mappings=hdr("s2v")),
                              T.FieldDescriptor(2, "w", T.builtin("string"), T.REQUIRED, http_mappings=hdr("s2w"))])
    s = T.struct_type("S", [T.FieldDescriptor(1, "a", T.builtin("string"), http_mappings=hdr("a")),
                            T.FieldDescriptor(2, "b", T.builtin("byte"), T.OPTIONAL, http_mappings=[("api.cookie", "b")]),
                            T.FieldDescriptor(3, "x", s2, http_mappings=hdr("x")),
                            T.FieldDescriptor(4, "r", T.builtin("string"), T.REQUIRED,
                                              http_mappings=[("api.raw_body", "")]),
                            T.FieldDescriptor(5, "n", T.builtin("i64"))])
    return T.struct_type("R", [
        T.FieldDescriptor(1, "h", T.builtin("string"), http_mappings=hdr("h")),
        T.FieldDescriptor(2, "c", T.builtin("i32"), http_mappings=[("api.http_code", "")]),
        T.FieldDescriptor(3, "s", s, http_mappings=[("api.cookie", "s")]),
        T.FieldDescriptor(4, "t", s),
        T.FieldDescriptor(5, "l", T.list_of(s), T.OPTIONAL),
        T.FieldDescriptor(6, "m", T.map_of(T.builtin("string"), s), T.OPTIONAL),
        T.FieldDescriptor(7, "d", T.builtin("double"), T.REQUIRED, http_mappings=hdr("d")),
        T.FieldDescriptor(8, "q", T.builtin("i64"), T.OPTIONAL, http_mappings=[("api.query", "q")]),
        T.FieldDescriptor(9, "k", T.list_of(T.builtin("i32")), http_mappings=hdr("k"))])


def test_hm_stops_vs_harness(chk):
    """Random messages (and mutated ones) under DG_T2J_HM, answered at
    random (taken / write as well / open for the JSON) call after call: at
    every step the device's status word and record (or final JSON) equal the
    harness's for the same answers."""
    td = hm_desc()
    fl = T.flatten(td)
    side = T.flatten_t2j(fl)
    rng = random.Random(11)
    msgs = [t2jgen.gen_thrift(rng, td) for _ in range(500)]
    msgs += [t2jgen.mutate(rng, t2jgen.gen_thrift(rng, td)) for _ in range(200)]
    seen = {"k1": 0, "k2": 0, "open": 0, "done": 0, "final": 0}
    for opts in (HM, HM | WDEF | WREQ | WOPT, HM | NOB64 | B8 | DISALLOW):
        answers = [bytearray() for _ in msgs]
        live = list(range(len(msgs)))
        for _step in range(60):
            if not live:
                break
            outs, rets = gpu_t2j_ans(fl, [msgs[i] for i in live], opts, [answers[i] for i in live])
            nxt = []
            for k, i in enumerate(live):
                er, eo, _ = chk.t2j3(fl, side, msgs[i], opts, bytes(answers[i]))
                assert (int(rets[k]), outs[k]) == (er, eo), (i, hex(int(rets[k])), hex(er), outs[k][-40:],
                                                            eo[-40:], bytes(answers[i]), msgs[i][:60].hex())
                if (er & 0xFF) != 12:
                    seen["final"] += 1
                    continue
                w0 = struct.unpack_from("<Q", eo, len(eo) - 16)[0]
                kind, idx, fi = w0 & 0xFF, (w0 >> 16) & 0xFFFF, w0 >> 32
                an = answers[i]
                if idx < len(an) and an[idx] == 2:
                    seen["done"] += 1
                    del an[idx:]
                    an.append(rng.randrange(2))
                else:
                    assert idx == len(an)
                    seen["k%d" % kind] += 1
                    container = fl.fields[fi].type.type in (T.STRUCT, T.MAP, T.LIST, T.SET)
                    if kind == 1 and container and rng.random() < 0.6:
                        seen["open"] += 1
                        an.append(2)
                    else:
                        an.append(rng.randrange(2))
                nxt.append(i)
            live = nxt
        assert not live
    assert min(seen.values()) > 20, seen


@pytest.mark.parametrize("name", ["test_http_mapping_fallback", "test_write_empty", "test_nobody_required_fields",
                                  "test_json_string", "test_kitex_api_header", "test_default_value",
                                  "test_optional_default_value", "test_conv_thrift2http", "test_errors",
                                  "test_http_conv"])
def test_reference_http_mapping_cases(chk, monkeypatch, name):
    """The reference's t2j HTTP-mapping tests (tests/test_t2j_http.py, there
    over the harness) with the GPU doing the conversion."""
    import inspect
    import test_t2j_http as th
    monkeypatch.setattr(th, "harness_conv", lambda _chk, o: t2j.BinaryConv(o))
    fn = getattr(th, name)
    if "nob64" in inspect.signature(fn).parameters:
        for v in (False, True):
            fn(chk, v)
    elif "use_default" in inspect.signature(fn).parameters:
        for v in (True, False):
            fn(chk, v)
    else:
        fn(chk)


def test_reference_known_answers_more(chk):
    """conv/t2j/conv_test.go's TestAPIBody (:288-308), TestUnknowFields
    (:472-518) and TestSimpleArgs (:711-733) through BinaryConv on the GPU,
    each also against the checker."""
    from test_t2j_oracle import API_BODY_JSON, _example3_resp_bin, _example3_svc, api_body_thrift
    fns = _example3_svc().functions()
    td = fns["ApiBodyMethod"].response().struct.fields[0].type
    assert t2j.BinaryConv(conv.Options(EnableValueMapping=True)).do(td, api_body_thrift()) == API_BODY_JSON
    assert not compare(chk, T.flatten(td), [api_body_thrift()], VM)
    src = _example3_resp_bin()
    for td in (fns["PartialMethod"].response().struct.fields[0].type,
               fns["PartialMethod"].request().struct.fields[0].type):
        with pytest.raises(t2j.T2JError) as ei:
            t2j.BinaryConv(conv.Options(DisallowUnknownField=True)).do(td, src)
        assert ei.value.behavior == "ErrUnknownField"
        t2j.BinaryConv(conv.Options()).do(td, src)
        assert not compare(chk, T.flatten(td), [src], DISALLOW)
        assert not compare(chk, T.flatten(td), [src], 0)
    for name, src, want in (("String", struct.pack(">i", 5) + b"hello", b'"hello"'),
                            ("I64", struct.pack(">q", 2**63 - 1), b"9223372036854775807")):
        td = fns[name].response().struct.fields[0].type
        assert t2j.BinaryConv(conv.Options()).do(td, src) == want
