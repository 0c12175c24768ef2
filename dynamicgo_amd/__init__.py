"""dynamicgo_amd — MI355X-native batched JSON -> Thrift-binary transcoder.

A drop-in for the hot path of cloudwego/dynamicgo's ``conv/j2t`` (BinaryConv.Do,
native j2t_fsm_exec). The compute lives in hand-written HIP kernels for gfx950
(dynamicgo_amd/csrc), exposed through a C ABI (include/dgj2t.h); this package is
the host-side mirror of the reference's Go API used by tests and bench.py.
"""
from . import thrift  # noqa: F401
from .thrift import (FlatDescriptor, Options as ThriftOptions, TypeDescriptor,  # noqa: F401
                     flatten, new_descriptor_by_name, new_descriptor_from_content,
                     new_descriptor_from_path)

__all__ = ["thrift", "flatten", "FlatDescriptor", "TypeDescriptor", "ThriftOptions",
           "new_descriptor_from_path", "new_descriptor_from_content", "new_descriptor_by_name"]
