"""CPU: the product library builds, loads, and exports every symbol that
include/dgj2t.h declares (no compute calls without a GPU)."""
import os
import re

from dynamicgo_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "dgj2t.h")).read()
    return sorted(set(re.findall(r"^[a-z_ 0-9*]+?\b(dg_[a-z0-9_]+)\(", txt, re.M)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_all_symbols():
    L = _lib.lib()
    for s in declared_symbols():
        assert hasattr(L, s), s


def test_slot_bound():
    assert _lib.lib().dg_slot_bound(100) >= 400


def test_descriptor_blob_layout():
    import struct
    from dynamicgo_amd.workloads import simple_desc
    from dynamicgo_amd.thrift import flatten
    fl = flatten(simple_desc())
    hdr = struct.unpack("<16I", fl.blob[:64])
    assert hdr[0] == 0x31444744 and hdr[1] == 2 and hdr[2] == len(fl.blob)
    assert hdr[4] >= 7 and hdr[6] == 1 and hdr[8] == 6  # types, 1 struct, 6 fields
