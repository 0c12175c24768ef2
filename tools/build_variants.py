"""Build experiment variants of the library (wave / flat kernel knobs):
python tools/build_variants.py NAME=-DFLAG=..,-DFLAG=.. ...  -> dynamicgo_amd/libdgj2t_NAME.so"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamicgo_amd import build as b  # noqa: E402

for spec in sys.argv[1:]:
    name, flags = spec.split("=", 1)
    fl = tuple(flags.split(","))
    out = os.path.join(b.ROOT, "dynamicgo_amd", f"libdgj2t_{name}.so")
    if all(f.startswith("-DDG_FL_") for f in fl):
        units = ("j2t_kern_flat.hip", "j2t_host.hip")
    elif all(f.startswith(("-DDG_T2W", "-DDG_T2J")) for f in fl):
        units = ("t2j_kern.hip",)
    elif all(f.startswith("-DDG_GW") for f in fl):
        units = ("j2t_pipe.hip",)
    else:
        units = ("j2t_kern_wave.hip", "j2t_kern_wave5.hip", "j2t_host.hip", "j2t_kern_flat.hip")
    b.build_hip(out=out, unit_flags={u: fl for u in units})
    print("built", out, flush=True)
