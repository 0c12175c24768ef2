"""Seeded random JSON generators for parity tests.

``gen_value(rng, td)`` produces JSON text that mostly matches the descriptor
(with deliberate type slips, nulls, unknown keys, escapes, odd numbers and
base64 corner cases); ``mutate`` damages it to reach the error paths.
"""
import base64
import random
import struct

from dynamicgo_amd import thrift as T

NUM_FORMS = [
    "0", "-0", "1", "-1", "01", "-01", "1.0", "1.5e-3", "1e400", "-1e400", "1E5", "1e+5", "1e-5",
    "0.1", "0.000001", "123456789012345678901234567890e-10", "9223372036854775807",
    "9223372036854775808", "-9223372036854775808", "-9223372036854775809",
    "99999999999999999999", "1.7976931348623157e+308", "4.9e-324", "2.2250738585072014e-308",
    "1e-400", "1.", "1.e5", "-", "--1", "1e", "1e+", "1.5.3", "1e5e5", "1+5", "0x10", "00",
    "1.9", "-1.9", "2147483647", "2147483648", "-2147483648", "-2147483649", "32767", "32768",
    "127", "128", "255", "256", "-129", "3.4028235e38", "7.0e-10", "0.30000000000000004",
    "179769313486231570000000000000000000000000000000000000000000000000000000000000000000000"
    "000000000000000000000000000000000000000000000000000000000000000000000000000000000000000"
    "000000000000000000000000000000000000000000000000000000000000000000000000000000000000000"
    "000000000000000000000000000000000000000000000000000000000000000000000000000.0",
    "2.4703282292062327e-324", "2.4703282292062328e-324", "1.00000000000000011102230246251565404236316680908203125",
    "9007199254740993", "9007199254740993.0", "123.456e7", "5e-324", "1e23", "8.98846567431158e307",
    "0.0000000000000000000000000000000000001", "1234567890123456789", "12345678901234567890",
    "1234567890.1234567890123", "-0.0", "0e0", "0E-0", "1e-0", "1e00000000000000000000001",
]
STR_PIECES = ["a", "b", "xyz", " ", "\\n", "\\t", "\\\\", "\\\"", "\\/", "\\u00e9", "\\u4e2d",
              "\\ud83d\\ude00", "\\ud800", "\\udc00", "\\uZZZZ", "\\x", "\\u12", "é", "中文",
              "\t", "\x01", "\\b", "\\f", "\\r", "\\u0000", "\\ud800\\u0041", "\\ud800x"]


def rnum(rng):
    r = rng.random()
    if r < 0.5:
        return rng.choice(NUM_FORMS)
    if r < 0.7:
        return str(rng.randint(-2**63, 2**63 - 1))
    if r < 0.8:
        return str(rng.randint(-300, 300))
    if r < 0.9:
        return repr(rng.uniform(-1e6, 1e6))
    return "%.17g" % (rng.random() * 10 ** rng.randint(-320, 308))


def rstr(rng, maxn=6):
    return '"' + "".join(rng.choice(STR_PIECES) for _ in range(rng.randint(0, maxn))) + '"'


def rb64(rng):
    r = rng.random()
    if r < 0.7:
        return '"' + base64.b64encode(bytes(rng.randrange(256) for _ in range(rng.randint(0, 20)))).decode() + '"'
    return '"' + rng.choice(["", "=", "==", "a", "ab", "abc", "abcd", "ab==", "abc=", "a===",
                             "QUJD\\n", "QUJD==", "QU\\r\\nJD", "QUJD\n", "Q\nUJD", "////", "-_-_",
                             "QUJ", "QQ=", "QQ==x", "aGk=\\n", "\\/\\/\\/\\/"]) + '"'


def gen_value(rng, td, depth=0):
    """JSON text (str) for a value of type ``td``."""
    if rng.random() < 0.04:
        return "null"
    if rng.random() < 0.03:  # type slip
        return rng.choice(["true", "false", "[]", "{}", '"s"', "1", "[1]", '{"a":1}', "nul", "tru"])
    t = td.type
    if t == T.BOOL:
        return rng.choice(["true", "false"])
    if t in (T.BYTE, T.I16, T.I32, T.I64, T.DOUBLE):
        if rng.random() < 0.08:
            return '"' + rnum(rng) + '"'
        return rnum(rng)
    if t == T.STRING:
        if td.is_binary():
            return rb64(rng)
        return rstr(rng)
    if t in (T.LIST, T.SET):
        if depth > 5:
            return "[]"
        n = rng.randint(0, 4)
        return "[" + ",".join(gen_value(rng, td.elem, depth + 1) for _ in range(n)) + "]"
    if t == T.MAP:
        if depth > 5:
            return "{}"
        n = rng.randint(0, 4)
        items = []
        for _ in range(n):
            if td.key.type == T.STRING:
                k = rstr(rng, 3)
            else:
                k = '"' + rng.choice([rnum(rng), rnum(rng), "12abc", "", "x", "-", "1 "]) + '"'
            items.append(k + ":" + gen_value(rng, td.elem, depth + 1))
        return "{" + ",".join(items) + "}"
    if t == T.STRUCT:
        if depth > 5:
            return "{}"
        sd = td.struct
        keys = list(sd.names.keys())
        items = []
        for _ in range(rng.randint(0, len(sd.fields) + 2)):
            r = rng.random()
            if r < 0.85 and keys:
                k = rng.choice(keys)
                f = sd.names[k]
                kj = '"' + k + '"'
                if rng.random() < 0.05 and k:
                    kj = '"' + "\\u%04x" % ord(k[0]) + k[1:] + '"'
                items.append(kj + ":" + gen_value(rng, f.type, depth + 1))
            else:
                items.append(rstr(rng, 2) + ":" + gen_any(rng, depth + 1))
        return "{" + ",".join(items) + "}"
    return "null"


def gen_any(rng, depth=0):
    r = rng.random()
    if depth > 4 or r < 0.3:
        return rnum(rng)
    if r < 0.5:
        return rstr(rng)
    if r < 0.6:
        return rng.choice(["true", "false", "null"])
    if r < 0.8:
        return "[" + ",".join(gen_any(rng, depth + 1) for _ in range(rng.randint(0, 3))) + "]"
    return "{" + ",".join(rstr(rng, 2) + ":" + gen_any(rng, depth + 1)
                         for _ in range(rng.randint(0, 3))) + "}"


def spacify(rng, s):
    if rng.random() < 0.7:
        return s
    out = []
    for ch in s:
        out.append(ch)
        if ch in ",:{}[]" and rng.random() < 0.3:
            out.append(rng.choice([" ", "\n", "\t  ", "\r\n", "     "]))
    return "".join(out)


def mutate(rng, b: bytes) -> bytes:
    if not b or rng.random() < 0.6:
        return b
    b = bytearray(b)
    for _ in range(rng.randint(1, 3)):
        op = rng.random()
        i = rng.randrange(len(b) + 1)
        if op < 0.3 and len(b) > 1:
            del b[i:i + rng.randint(1, 3)]
        elif op < 0.6:
            b[i:i] = rng.choice([b",", b"}", b"]", b'"', b"\\", b" ", b"x", b"0", b"-", b"{", b"["])
        elif op < 0.8 and i < len(b):
            b[i] = rng.randrange(256)
        else:
            b = b[:i]
    return bytes(b)


def gen_message(rng, td, mutate_p=True) -> bytes:
    s = spacify(rng, gen_value(rng, td))
    if rng.random() < 0.05:
        s = s + rng.choice([" ", " xyz", "\n\n\n\n\n", "}", "  \t"])
    b = s.encode()
    return mutate(rng, b) if mutate_p else b
