"""CPU: the oracle restatement against the reference-generated golden vectors
(and against the reference engine itself when oracle/_ref is built)."""
import random

import pytest

import oracle
import fuzz
from dynamicgo_amd import thrift as T, workloads as W
from schemas import probe, idl_desc


def test_port_oracle_matches_golden(golden):
    rows, flats = golden
    port = oracle.PortOracle()
    bad = []
    for name, flags, js, ret, out in rows:
        r, o = port.j2t(flats[name], js, flags)
        if r != ret or o != out:
            bad.append((name, flags, js[:80], hex(r), hex(ret)))
    assert not bad, bad[:5]


def test_ref_oracle_matches_golden(golden):
    ref = oracle.RefOracle()
    if ref is None:
        pytest.skip("oracle/_ref not built")
    rows, flats = golden
    for name, flags, js, ret, out in rows:
        r, o = ref.j2t(flats[name], js, flags)
        assert (r, o) == (ret, out), (name, flags, js[:80])


def test_appendix_d_known_answers(golden):
    """SURVEY.md Appendix D vectors, captured from the reference engine."""
    rows, _ = golden
    want = {
        b'{"A":1,"A":2}': (0, "080001000000010800010000000200"),
        b'{"D":"xxx"}': (0x30000000a0e, ""),
        b'{"A":01}': (0x31020000000702, ""),
        b'{"E":1e400}': (0x50000000a08, ""),
        b'{"C":[1.0e2, -9223372036854775808, 9223372036854775808]}':
            (0, "0f00030a0000000300000000000000648000000000000000800000000000000000"),
        b'{"A":"7"}': (0, "06000100070700"),
    }
    got = {js: (ret, out.hex()) for _, _, js, ret, out in rows if js in want}
    assert got == want


def test_reference_payload_sizes(golden):
    """introduction.md:101,103 — Simple 114 B, Nesting 6455 B of Thrift."""
    rows, _ = golden
    sizes = {(n, len(js)): len(out) for n, f, js, r, out in rows if n in ("simple", "nesting") and f == 1 and r == 0}
    assert sizes[("simple", 236)] == 114
    assert sizes[("nesting", 11855)] == 6455


@pytest.mark.parametrize("seed", [11, 12])
def test_port_vs_reference_fuzz(seed):
    ref = oracle.RefOracle()
    if ref is None:
        pytest.skip("oracle/_ref not built")
    port = oracle.PortOracle()
    rng = random.Random(seed)
    for td in (probe("D2"), idl_desc("baseline.thrift", "NestingMethod"), idl_desc("example3.thrift", "ExampleMethod")):
        fl = T.flatten(td)
        for _ in range(400):
            m = fuzz.gen_message(rng, td)
            flags = rng.choice([1, 0, 0x11, 0x5, 0x23, 0x83])
            assert ref.j2t(fl, m, flags) == port.j2t(fl, m, flags), (m, flags)


UTF8_FLAG = 1 << 16  # DG_F_VALIDATE_UTF8 (extension; no reference counterpart)

UTF8_CASES = [  # (string body bytes, offset of the first invalid sequence or None)
    (b"abc", None), ("é中文😀".encode(), None), (b"a\\u00e9\\n", None), (b"", None),
    (b"a\xff", 1), (b"\xc0\x80", 0), (b"\xc1\xbf", 0), (b"\xed\xa0\x80", 0), (b"\xe0\x80\x80", 0),
    (b"\xf0\x80\x80\x80", 0), (b"\xf4\x90\x80\x80", 0), (b"\xf5\x80\x80\x80", 0), (b"xy\xe4\xb8", 2),
    (b"\xe4\xb8\xad\x80", 3), (b"12345678\xc3", 8), (b"\xef\xbf\xbf", None), (b"\xf4\x8f\xbf\xbf", None),
]


def _pack(code, value, pos):
    return ((value << 40) | (pos << 8) | code) & (2**64 - 1)


@pytest.mark.parametrize("body,bad", UTF8_CASES)
def test_utf8_validation_extension(body, bad):
    """DG_F_VALIDATE_UTF8 on the port oracle: valid strings convert exactly as
    without the flag; the first invalid sequence (utf8_validate semantics,
    native/utf8.c:101-212) gives ERR_INVAL at its offset. The reference has no
    such flag; the verdicts are pinned to its own validator by
    test_utf8_extension_pinned_to_reference_validator below."""
    chk = oracle.PortOracle()
    fl = T.flatten(idl_desc("baseline.thrift", "SimpleMethod"))
    pre = b'{"StringField":"'
    msg = pre + body + b'"}'
    r0 = chk.j2t(fl, msg, 1)
    r1 = chk.j2t(fl, msg, 1 | UTF8_FLAG)
    if bad is None:
        assert r1 == r0
    else:
        assert r1 == (_pack(2, body[bad], len(pre) + bad), b"")
    # binary fields are base64 text, not validated
    assert chk.j2t(fl, b'{"BinaryField":"\xff"}', 1 | UTF8_FLAG) == chk.j2t(fl, b'{"BinaryField":"\xff"}', 1)


def utf8_fuzz_bodies(seed: int, n: int):
    """JSON string bodies (no raw '"' or '\\') mixing valid UTF-8, ASCII,
    escapes and invalid sequences: truncated, overlong, surrogate, out of
    range, stray continuation bytes."""
    rng = random.Random(seed)
    pieces = [b"a", b"Z0", b" ", b"\\n", b"\\u00e9", "é".encode(), "中".encode(), "😀".encode(), b"\xc3", b"\xe4\xb8",
              b"\xf0\x9f\x98", b"\x80", b"\xbf", b"\xc0\x80", b"\xc1\xbf", b"\xe0\x9f\xbf", b"\xed\xa0\x80",
              b"\xf0\x8f\xbf\xbf", b"\xf4\x90\x80\x80", b"\xf5\x80\x80\x80", b"\xff", b"\x01\x1f", b"\xef\xbf\xbf",
              b"\xf4\x8f\xbf\xbf", b"\xe0\xa0\x80", b"\xed\x9f\xbf", b"0123456789abcdefXYZ"]
    out = []
    for _ in range(n):
        if rng.random() < 0.3:  # raw random bytes
            b = bytes(rng.choice([c for c in range(256) if c not in (0x22, 0x5C)]) for _ in range(rng.randint(0, 40)))
        else:
            b = b"".join(rng.choice(pieces) for _ in range(rng.randint(0, 14)))
        out.append(b)
    return out


def test_utf8_extension_pinned_to_reference_validator():
    """the DG_F_VALIDATE_UTF8 verdicts pinned to the
    reference's own validator, utf8_validate (native/utf8.c:183-212, compiled
    from /root/reference into oracle/_ref): on the table above and 3 000
    fuzz bodies, a string is rejected exactly when utf8_validate returns an
    offset, with ERR_INVAL at that byte; otherwise the output is the
    reference's flag-off output."""
    if oracle.RefOracle() is None:
        pytest.skip("oracle/_ref not built")
    for body, bad in UTF8_CASES:
        assert oracle.ref_utf8_validate(body) == (-1 if bad is None else bad), body
    ref = oracle.RefOracle()
    port = oracle.PortOracle()
    fl = T.flatten(idl_desc("baseline.thrift", "SimpleMethod"))
    pre = b'{"StringField":"'
    n_bad = 0
    for body in UTF8_CASES_BODIES + utf8_fuzz_bodies(61, 3000):
        msg = pre + body + b'"}'
        bad = oracle.ref_utf8_validate(body)
        want = ref.j2t(fl, msg, 1) if bad < 0 else (_pack(2, body[bad], len(pre) + bad), b"")
        n_bad += bad >= 0
        assert port.j2t(fl, msg, 1 | UTF8_FLAG) == want, body
    assert 300 < n_bad < 2900


UTF8_CASES_BODIES = [b for b, _ in UTF8_CASES]


def test_unterminated_string_block_tail():
    """The one malformed-input class where the reference's verdict is
    undefined: an unterminated string whose bytes after the opening quote end
    exactly at a SIMD block boundary. advance_string (native/scanning.c:130-375)
    then skips its scalar tail loop and tests `if (ch == '"')` on an
    uninitialised `ch` (declared at :132, only assigned inside the loop at
    :342). The restatement (and the GPU) report ERR_EOF at the end, as for
    every other unterminated string; whatever the compiled reference returns
    there depends on a stale register. Any other tail length agrees."""
    ref = oracle.RefOracle()
    port = oracle.PortOracle()
    fl = T.flatten(probe("D3"))
    for k in range(1, 70):
        m = b'{"x":1,"y":"' + b"a" * k
        r, _ = port.j2t(fl, m, 1)
        assert r & 0xFF == 1 and (r >> 8) & 0xFFFFFFFF == len(m), (k, hex(r))  # ERR_EOF at len
        if ref is not None and k % 32:
            assert ref.j2t(fl, m, 1)[0] == r, k


def test_batch_wrapper_redoes_outputs_larger_than_their_slot():
    """j2t_batch sizes slots at 4x the message + 64; default writes of a tiny
    message outgrow that ("{}" of NestingI64 with WRITE_DEFAULT: 120 bytes),
    and the harness then reports the full length without the bytes. The
    wrapper converts such messages again alone (found by tools/fuzz_sweep.py:
    the batch checker returned zeros where the GPU was right)."""
    fl = T.flatten(W.nesting_i64_desc())
    msgs = [b"{}", b'{"I32":5}', b"{}"]
    for o in [x for x in (oracle.RefOracle(), oracle.PortOracle()) if x]:
        for flags in (0x2, 0x3, 0x7):
            er, eo = o.j2t_batch(fl, msgs, flags)
            want = [o.j2t(fl, m, flags) for m in msgs]
            assert [(int(r), b) for r, b in zip(er, eo)] == want
            assert all(len(b) > 4 * 2 + 64 for b in eo)
