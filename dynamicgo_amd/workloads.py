"""Synthetic workloads of BASELINE.json's configs.

  C1  the reference's Simple payload (testdata/test/baseline_j2t_test.go:116-125),
      Go encoding/json form: 236 B JSON -> 114 B Thrift
  C2  65 536 flat `baseline.Simple` messages <= 256 B, seed 42
  C3  65 536 nested `NestingI64` messages (baseline.Nesting with field 15 as
      map<i64, Simple>), seed 43
  C4  4 096 large messages {1: binary Blob, 2: list<double> Values, 3: string Name},
      48 KiB base64 blob + 1024 doubles each (~90 KiB), seed 44
  C5  1 048 576 messages: 90 % C2-like / 9.5 % C3-like / 0.5 % C4-like, seed 45
      (mixed-schema: each message carries its own root in a wrapper struct)

Descriptors are built from the reference's IDL text (baseline.thrift), parsed
by dynamicgo_amd.thrift. All data is synthetic (no network, no datasets).
"""
from __future__ import annotations

import base64
import random
from typing import List

import numpy as np

from . import thrift as T

BASELINE_IDL = """
namespace go baseline
struct Simple {
    1: byte ByteField
    2: i64 I64Field (api.js_conv = "")
    3: double DoubleField
    4: i32 I32Field
    5: string StringField,
    6: binary BinaryField
}
struct Nesting {
    1: string String (api.header = "String")
    2: list<Simple> ListSimple
    3: double Double (api.path = "double")
    4: i32 I32 (api.http_code = "", api.body = "I32")
    5: list<i32> ListI32 (api.query = "ListI32")
    6: i64 I64
    7: map<string, string> MapStringString
    8: Simple SimpleStruct
    9: map<i32, i64> MapI32I64
    10: list<string> ListString
    11: binary Binary
    12: map<i64, string> MapI64String
    13: list<i64> ListI64 (api.cookie = "list_i64"),
    14: byte Byte
    15: map<string, Simple> MapStringSimple
}
struct NestingI64 {
    1: string String (api.header = "String")
    2: list<Simple> ListSimple
    3: double Double (api.path = "double")
    4: i32 I32 (api.http_code = "", api.body = "I32")
    5: list<i32> ListI32 (api.query = "ListI32")
    6: i64 I64
    7: map<string, string> MapStringString
    8: Simple SimpleStruct
    9: map<i32, i64> MapI32I64
    10: list<string> ListString
    11: binary Binary
    12: map<i64, string> MapI64String
    13: list<i64> ListI64 (api.cookie = "list_i64"),
    14: byte Byte
    15: map<i64, Simple> MapStringSimple
}
struct Large {
    1: binary Blob
    2: list<double> Values
    3: string Name
}
struct Mixed {
    1: Simple Flat
    2: NestingI64 Nested
    3: Large Big
}
"""


def _desc(name: str) -> T.TypeDescriptor:
    return T.new_descriptor_by_name("baseline.thrift", BASELINE_IDL, name)


def simple_desc():
    return _desc("Simple")


def nesting_desc():
    return _desc("Nesting")


def nesting_i64_desc():
    return _desc("NestingI64")


def large_desc():
    return _desc("Large")


def mixed_desc():
    return _desc("Mixed")


def go_json_string(s: str) -> str:
    """encoding/json string encoding (HTML-safe escaping, \\u0008 for \\b)."""
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif o < 0x20 or ch in "<>&" or o in (0x2028, 0x2029):
            out.append("\\u%04x" % o)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def c1_simple_json() -> bytes:
    """The reference's Simple sample (baseline_j2t_test.go:108-125)."""
    s = "你好,\b\n\r\t世界" * 2
    b = bytes(range(16)) * 2
    return ('{"ByteField":127,"I64Field":9223372036854775807,"DoubleField":1.7976931348623157e+308,'
            '"I32Field":2147483647,"StringField":%s,"BinaryField":"%s"}'
            % (go_json_string(s), base64.b64encode(b).decode())).encode()


_ALNUM = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789 _-.,"


def _rstring(rng: random.Random) -> str:
    n = rng.randint(0, 48)
    s = "".join(rng.choice(_ALNUM) for _ in range(n))
    if rng.random() < 0.1:
        esc = rng.choice(["\\n", "\\u00e9"])
        k = rng.randint(0, len(s))
        s = s[:k] + esc + s[k:]
    return '"' + s + '"'


def _rdouble(rng: random.Random) -> str:
    if rng.random() < 0.5:
        v = round(rng.uniform(-1e4, 1e4), rng.randint(0, 2))
        return ("%.6g" % v)
    return "%.17g" % rng.uniform(-1e6, 1e6)


def simple_obj(rng: random.Random) -> str:
    return ('{"ByteField":%d,"I64Field":%d,"DoubleField":%s,"I32Field":%d,"StringField":%s,"BinaryField":"%s"}'
            % (rng.randint(-128, 127), rng.randint(-2**63, 2**63 - 1), _rdouble(rng),
               rng.randint(-2**31, 2**31 - 1), _rstring(rng),
               base64.b64encode(rng.randbytes(rng.randint(0, 60))).decode()))


def gen_flat_batch(rng: random.Random, n: int, max_len: int = 256) -> List[bytes]:
    """C2: flat Simple messages, each <= max_len bytes (redraw if longer)."""
    out = []
    while len(out) < n:
        m = simple_obj(rng).encode()
        if len(m) <= max_len:
            out.append(m)
    return out


def nesting_obj(rng: random.Random) -> str:
    ls = ",".join(simple_obj(rng) for _ in range(rng.randint(0, 8)))
    li32 = ",".join(str(rng.randint(-2**31, 2**31 - 1)) for _ in range(rng.randint(0, 8)))
    mss = ",".join('"k%d":%s' % (i, _rstring(rng)) for i in range(rng.randint(0, 4)))
    mi32 = ",".join('"%d":%d' % (rng.randint(-2**31, 2**31 - 1), rng.randint(-2**63, 2**63 - 1))
                    for _ in range(rng.randint(0, 4)))
    lstr = ",".join(_rstring(rng) for _ in range(rng.randint(0, 8)))
    mi64s = ",".join('"%d":%s' % (rng.randint(-2**63, 2**63 - 1), _rstring(rng)) for _ in range(rng.randint(0, 4)))
    li64 = ",".join(str(rng.randint(-2**63, 2**63 - 1)) for _ in range(rng.randint(0, 8)))
    mis = ",".join('"%d":%s' % (rng.randint(-2**63, 2**63 - 1), simple_obj(rng)) for _ in range(rng.randint(0, 4)))
    return ('{"String":%s,"ListSimple":[%s],"Double":%s,"I32":%d,"ListI32":[%s],"I64":%d,'
            '"MapStringString":{%s},"SimpleStruct":%s,"MapI32I64":{%s},"ListString":[%s],'
            '"Binary":"%s","MapI64String":{%s},"ListI64":[%s],"Byte":%d,"MapStringSimple":{%s}}'
            % (_rstring(rng), ls, _rdouble(rng), rng.randint(-2**31, 2**31 - 1), li32,
               rng.randint(-2**63, 2**63 - 1), mss, simple_obj(rng), mi32, lstr,
               base64.b64encode(rng.randbytes(rng.randint(0, 60))).decode(), mi64s, li64,
               rng.randint(-128, 127), mis))


def gen_nested_batch(rng: random.Random, n: int) -> List[bytes]:
    """C3: NestingI64 messages."""
    return [nesting_obj(rng).encode() for _ in range(n)]


def large_obj(rng: random.Random, blob_bytes: int = 48 * 1024, n_values: int = 1024) -> bytes:
    nr = np.random.default_rng(rng.getrandbits(64))
    blob = base64.b64encode(nr.bytes(blob_bytes))
    vals = nr.uniform(-1e6, 1e6, n_values)
    vs = ",".join("%.17g" % v for v in vals.tolist())
    return b'{"Blob":"' + blob + b'","Values":[' + vs.encode() + b'],"Name":' + _rstring(rng).encode() + b"}"


def gen_large_batch(rng: random.Random, n: int, blob_bytes: int = 48 * 1024, n_values: int = 1024) -> List[bytes]:
    """C4: large messages (>= 64 KiB JSON each at the default sizes)."""
    return [large_obj(rng, blob_bytes, n_values) for _ in range(n)]


def gen_mixed_batch(rng: random.Random, n: int, large_scale: float = 1.0) -> List[bytes]:
    """C5: 90 % flat / 9.5 % nested / 0.5 % large, each wrapped as one field of Mixed."""
    out = []
    for _ in range(n):
        r = rng.random()
        if r < 0.9:
            out.append(b'{"Flat":' + simple_obj(rng).encode() + b"}")
        elif r < 0.995:
            out.append(b'{"Nested":' + nesting_obj(rng).encode() + b"}")
        else:
            out.append(b'{"Big":' + large_obj(rng, int(48 * 1024 * large_scale), int(1024 * large_scale)) + b"}")
    return out


def arena(msgs: List[bytes], pad: int = 64):
    """(uint8 arena with `pad` zero bytes, uint64 offsets[n+1])."""
    lens = np.fromiter((len(m) for m in msgs), dtype=np.uint64, count=len(msgs))
    off = np.zeros(len(msgs) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    a = np.frombuffer(b"".join(msgs) + b"\0" * pad, dtype=np.uint8).copy()
    return a, off


# ---- C5 as ONE global batch: chunk-seeded so that it can be
# generated in parallel and identically on every rank ----
C5_MESSAGES = 1 << 20
C5_CHUNK = 16384


def _mixed_chunk(args):
    seed, c, n, large_scale = args
    msgs = gen_mixed_batch(random.Random(seed * 1_000_003 + c), n, large_scale)
    return b"".join(msgs), np.fromiter((len(m) for m in msgs), dtype=np.uint64, count=len(msgs))


def gen_mixed_arena(n: int = C5_MESSAGES, seed: int = 45, workers: int = 1, large_scale: float = 1.0,
                    chunk: int = C5_CHUNK, pad: int = 64):
    """C5: n mixed messages as (arena, offsets[n+1]). Message block c (chunk
    messages each) draws from Random(seed * 1000003 + c), so the batch is the
    same whatever the worker count; workers > 1 uses a fork pool (call before
    anything initialises the GPU)."""
    jobs = [(seed, c, min(chunk, n - c * chunk), large_scale) for c in range((n + chunk - 1) // chunk)]
    if workers > 1 and len(jobs) > 1:
        import multiprocessing as mp
        with mp.get_context("fork").Pool(min(workers, len(jobs))) as pool:
            parts = pool.map(_mixed_chunk, jobs)
    else:
        parts = [_mixed_chunk(j) for j in jobs]
    lens = np.concatenate([p[1] for p in parts]) if parts else np.zeros(0, dtype=np.uint64)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    a = np.empty(int(off[-1]) + pad, dtype=np.uint8)
    pos = 0
    for blob, _ in parts:
        a[pos:pos + len(blob)] = np.frombuffer(blob, dtype=np.uint8)
        pos += len(blob)
    a[pos:] = 0
    return a, off


def arena_slice(a: np.ndarray, off: np.ndarray, lo: int, hi: int, pad: int = 64):
    """Messages [lo, hi) of an arena as their own (arena, offsets) pair."""
    s, e = int(off[lo]), int(off[hi])
    sub = np.zeros(e - s + pad, dtype=np.uint8)
    sub[:e - s] = a[s:e]
    return sub, (off[lo:hi + 1] - off[lo]).astype(np.uint64)


def simple_obj_shuffled(rng: random.Random) -> str:
    """simple_obj with the six keys in a random order (C2's divergence
    stress, SURVEY.md §8(d): lanes of a wave no longer meet the same key)."""
    parts = ['"ByteField":%d' % rng.randint(-128, 127), '"I64Field":%d' % rng.randint(-2**63, 2**63 - 1),
             '"DoubleField":%s' % _rdouble(rng), '"I32Field":%d' % rng.randint(-2**31, 2**31 - 1),
             '"StringField":%s' % _rstring(rng),
             '"BinaryField":"%s"' % base64.b64encode(rng.randbytes(rng.randint(0, 60))).decode()]
    rng.shuffle(parts)
    return "{" + ",".join(parts) + "}"


def gen_flat_batch_shuffled(rng: random.Random, n: int, max_len: int = 256) -> List[bytes]:
    """C2 divergence stress: flat Simple messages with shuffled key order."""
    out = []
    while len(out) < n:
        m = simple_obj_shuffled(rng).encode()
        if len(m) <= max_len:
            out.append(m)
    return out
