import sys, os, random
sys.path[:0] = ['.', 'oracle', 'tests', 'tests/golden']
import numpy as np, torch
from dynamicgo_amd import conv, thrift as T, workloads as W, _lib
fn = T.new_descriptor_from_path('tests/golden/idl/baseline.thrift').functions()['SimpleMethod']
hc = conv.HTTPConv(conv.ENCODING_THRIFT_BINARY, fn)
bodies = W.gen_flat_batch(random.Random(5), 5)
outs, rets = hc.do_batch([conv.HTTPRequest(b) for b in bodies])
print([len(o) for o in outs], rets)
# non-framed scan on the same
cv = conv.BinaryConv(conv.Options(EnableHttpMapping=True)); ctx = cv._ctx(); flat = cv._flat(hc.st)
a, off = W.arena(bodies); n = len(bodies)
dev = torch.device('cuda:0')
slots = np.zeros(n + 1, dtype=np.int64); np.cumsum((np.diff(off).astype(np.int64) * 4 + 64 + 7) & ~7, out=slots[1:])
d_json = torch.from_numpy(a).to(dev); d_in = torch.from_numpy(off.astype(np.int64)).to(dev); d_oo = torch.from_numpy(slots).to(dev)
d_out = torch.zeros(int(slots[-1]) + 64, dtype=torch.uint8, device=dev); d_ol = torch.zeros(n, dtype=torch.int32, device=dev); d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
L = _lib.lib(); st = torch.cuda.current_stream()
_lib.check(L.dg_j2t_batch_device(ctx.h, ctx.desc(flat), flat.root_type, d_json.data_ptr(), d_in.data_ptr(), n, 9, d_out.data_ptr(), d_oo.data_ptr(), d_ol.data_ptr(), d_ret.data_ptr(), None, st.cuda_stream))
torch.cuda.synchronize(); print('ol', d_ol.cpu().tolist(), 'ret', d_ret.cpu().tolist())
d_dst = torch.zeros(int(slots[-1]) * 2 + 640, dtype=torch.uint8, device=dev); d_doff = torch.full((n + 1,), -1, dtype=torch.int64, device=dev)
_lib.check(L.dg_pack_device_scan(ctx.h, d_out.data_ptr(), d_oo.data_ptr(), d_ol.data_ptr(), n, d_dst.data_ptr(), d_doff.data_ptr(), st.cuda_stream))
torch.cuda.synchronize(); print('scan doff', d_doff.cpu().tolist())
d_doff.fill_(-1)
_lib.check(L.dg_pack_device_framed(ctx.h, d_out.data_ptr(), d_oo.data_ptr(), d_ol.data_ptr(), d_ret.data_ptr(), n, hc.top, len(hc.top), hc.bottom, len(hc.bottom), d_dst.data_ptr(), d_doff.data_ptr(), st.cuda_stream))
torch.cuda.synchronize(); print('framed doff', d_doff.cpu().tolist(), len(hc.top))
rng = random.Random(5)
bodies = W.gen_flat_batch(rng, 3000) + [b"{]", b"", b"{}", b'{"I32Field":tru}']
outs, rets = hc.do_batch([conv.HTTPRequest(b) for b in bodies])
bad = [i for i, (o, r) in enumerate(zip(outs, rets)) if r == 0 and not o]
print('n', len(bodies), 'bad', len(bad), bad[:10], bad[-3:] if bad else None, 'total', sum(len(o) for o in outs))
