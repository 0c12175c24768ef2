import sys; sys.path[:0]=['oracle','tests','tests/golden']
from schemas import idl_desc
from dynamicgo_amd import thrift as T
from test_gpu_parity import _raw_batch
td=idl_desc('baseline.thrift','NestingMethod'); fl=T.flatten(td)
for fl_ in (0x1|0x8|(1<<20), 0x1|0x8|(1<<20)|(1<<18), 0x1|0x8|(1<<20)|(1<<17), 0x1|0x8):
    print(hex(fl_), _raw_batch(fl, [b'{}', b'{"I64":5}'], fl_))
