"""GPU: the reference's mid-message callbacks served around the device
conversion -- non-inline value mapping (ERR_VM_END) and a nested struct's
ERR_HM_END -- against the reference's own FSM (oracle/_ref) with the same
host answers (oracle/vm_host.h, the Python handleUnmatchedFields through
dgref_set_hm_end_cb)."""
import random

import pytest

import oracle
import vm_maps
from dynamicgo_amd import conv, http as H, thrift as T
from schemas import idl_desc, vm_probe
from test_vm_oracle import AGW_DATA, agw_dynamic_body_expected, dynamic_struct, vm_message, _tstr, VM_CASES
import fuzz

pytestmark = pytest.mark.gpu
vm_maps.register()
REF = oracle.RefOracle()


def _agree(td, msgs, opts):
    """product (BinaryConv over the GPU) vs the reference FSM, message by
    message: same bytes, or the same status word; a host callback that failed
    is a ConvError on our side and the callback's stop word (ERR_VM_END) on
    the reference's."""
    fl = T.flatten(td)
    flags = conv.to_flags(opts)
    outs, errs = conv.BinaryConv(opts).do_batch_errors(td, msgs)
    n_ok = 0
    for m, o, e in zip(msgs, outs, errs):
        r, want = REF.j2t(fl, m, flags)
        if r == 0:
            assert e is None and o == want, (m, e)
            n_ok += 1
        elif r & 0xFF == 24:
            assert isinstance(e, H.ConvError), (m, e, hex(r))
        else:
            assert isinstance(e, conv.J2TError) and e.ret == r, (m, e, hex(r))
    return n_ok


def test_agw_dynamic_body_no_http_mapping():
    """TestAGWDynamicBody "no http-mapping" (conv/j2t/conv_test.go:931-946)."""
    opts = conv.Options(EnableValueMapping=True, WriteRequireField=True, ReadHttpValueFallback=True)
    td = dynamic_struct()
    out = conv.BinaryConv(opts).do(td, AGW_DATA)
    assert out == agw_dynamic_body_expected()
    assert REF.j2t(T.flatten(td), AGW_DATA, conv.to_flags(opts)) == (0, out)


def test_agw_dynamic_body_http_mapping():
    """TestAGWDynamicBody "http-mapping" (conv/j2t/conv_test.go:947-968):
    Query from the URL (api.query), the two body_dynamic values from the
    body, and the inner struct's required Must -- absent from the body --
    from the request (TracebackRequredOrRootFields, a NESTED ERR_HM_END)."""
    opts = conv.Options(EnableValueMapping=True, EnableHttpMapping=True, WriteRequireField=True,
                        ReadHttpValueFallback=True, TracebackRequredOrRootFields=True)
    td = dynamic_struct()
    data = '{"json":[1,2,3],"inner_struct":{"inner_json":{"a":"中文","b":1}}}'.encode()
    req = conv.HTTPRequest(b"", url="http://localhost?query=1&Must=2")
    out = conv.BinaryConv(opts).do(td, data, req=req)
    inner = b"\x0b\x00\x01" + _tstr('{"a":"中文","b":1}'.encode()) + b"\x0b\x00\x02" + _tstr(b"2") + b"\x00"
    assert out == (b"\x0b\x00\x01" + _tstr(b"1") + b"\x0b\x00\x02" + _tstr(b"[1,2,3]") +
                   b"\x0c\x00\x03" + inner + b"\x00")
    # the reference FSM with the same host half at both callbacks
    fl = T.flatten(td)
    hx = H.HMContext(opts, conv.BinaryConv(opts)._nested(conv.to_flags(opts)))
    ents = []
    for sd in fl.structs:
        ents.append(hx.handle_http_mappings(req, sd, False)[:2] if sd.hms else (b"", 0))
    REF.set_hm_end_cb(lambda si, ids: hx.handle_unmatched_fields(req, fl.structs[si], ids, True) + b"\x00")
    try:
        r, ref_out, _ = REF.j2t_hm3(fl, data, conv.to_flags(opts), ents)
    finally:
        REF.set_hm_end_cb(None)
    assert (r, ref_out) == (0, out)


def test_vm_cases():
    td = vm_probe()
    for flags_opts in (conv.Options(EnableValueMapping=True),
                       conv.Options(EnableValueMapping=True, WriteRequireField=True),
                       conv.Options(EnableValueMapping=True, WriteDefaultField=True),
                       conv.Options()):
        _agree(td, VM_CASES, flags_opts)


def test_vm_batch_vs_reference():
    """1 500 D4 messages in one batch: most callbacks served (several per
    message, at the root, in a nested struct and in list elements), some
    failing, some messages malformed."""
    rng = random.Random(9)
    td = vm_probe()
    msgs = [vm_message(rng) for _ in range(1000)] + [fuzz.gen_message(rng, td) for _ in range(500)]
    # a body_dynamic value deeper than the device's skip stack (the deep pass)
    msgs += [b'{"B":' + b"[" * 300 + b"]" * 300 + b',"A":"5"}', b'{"F":{"x":' + b'{"a":' * 100 + b"1" +
             b"}" * 100 + b',"y":1}}']
    assert _agree(td, msgs, conv.Options(EnableValueMapping=True)) > 700


def test_vm_example3_fuzz():
    """example3's body_dynamic fields (ExampleDynamicStruct) under fuzz."""
    rng = random.Random(10)
    td = dynamic_struct()
    msgs = [fuzz.gen_message(rng, td) for _ in range(600)]
    _agree(td, msgs, conv.Options(EnableValueMapping=True, WriteRequireField=True))


def test_many_callbacks_in_one_message_two_passes(monkeypatch):
    """a message with k non-inline value-mapping callbacks
    (ERR_VM_END, native/thrift.c:641-665) takes 2 device passes, not k + 1:
    DG_F_CB_COLLECT records every callback of a pass and converts on, the
    host serves them in message order, then one rerun writes the answers
    (the reference resumes its FSM in place, conv/j2t/impl_amd64.go:169-247).
    Messages with 64..400 callbacks -- list<struct> elements, duplicate root
    keys, a nested struct's own, a failing callback in the middle, a JSON
    error after the last callback -- agree with the reference FSM serving
    the same callbacks one by one."""
    td = vm_probe()
    rng = random.Random(64)
    msgs = [b'{"G":[' + b",".join(b'{"y":%d}' % rng.randint(-300, 300) for _ in range(n)) + b"]}"
            for n in (64, 100, 257, 400)]
    msgs.append(b"{" + b",".join(b'"A":"%d"' % k for k in range(80)) + b"}")
    msgs.append(b'{"G":[' + b",".join(b'{"y":"%d","x":[%d]}' % (k, k) for k in range(70)) + b'],"D":2.5}')
    bad = [b'{"y":%d}' % k for k in range(90)]
    bad[45] = b'{"y":"4x"}'  # JSConv2 rejects it: the error of the 46th callback
    msgs.append(b'{"G":[' + b",".join(bad) + b"]}")
    msgs.append(b'{"G":[' + b",".join(b'{"y":%d}' % k for k in range(66)) + b'],"C":[1,}')  # JSON error after them
    passes = []
    orig = conv.BinaryConv._host_cb

    def counted(self, *a, **kw):
        passes.append(len(a[1]))
        return orig(self, *a, **kw)
    monkeypatch.setattr(conv.BinaryConv, "_host_cb", counted)
    n_ok = _agree(td, msgs, conv.Options(EnableValueMapping=True))
    assert n_ok == 6
    assert len(passes) == 1, passes  # the main pass + ONE rerun for all callbacks of all messages
