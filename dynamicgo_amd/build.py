"""Build the in-tree native artefacts.

  dynamicgo_amd/libdgj2t.so        HIP kernels + C ABI for gfx950 (the product)
  oracle/_build/libj2t_oracle.so   plain-C restatement (test infrastructure)
  oracle/_ref/libdgref*.so         the reference's own native/*.c (test
                                   infrastructure; only when /root/reference exists)

Usage: python -m dynamicgo_amd.build [--no-oracle]
"""
import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dynamicgo_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("DG_OFFLOAD_ARCH", "gfx950")


def _run(cmd, cwd=None):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, cwd=cwd, check=True)


UNITS = ("j2t_kern_wave.hip", "j2t_kern_wave5.hip", "j2t_kern_small.hip", "j2t_kern_lds.hip", "j2t_kern_glb.hip",
         "j2t_host.hip", "j2t_pipe.hip", "t2j_kern.hip", "t2j_host.hip", "j2t_kern_flat.hip")
HEADERS = ("j2t_small.h", "j2t_wave.h", "j2t_machine.h", "j2t_device.h", "j2t_fast.h", "dg_tables.h", "host_internal.h",
           "t2j_device.h", "t2j_tables.h", "j2t_flat.h", "t2j_wave.h")


def source_hash(extra_flags=()) -> str:
    """sha256 over every source the library is built from, the compiler
    flags and the target arch: the library's identity."""
    h = hashlib.sha256()
    for f in sorted(UNITS + HEADERS):
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    for f in ("dgj2t.h", "dgj2t_defs.h", "dgj2t_desc.h"):
        with open(os.path.join(ROOT, "include", f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    h.update(repr((ARCH, COMMON_FLAGS, sorted(DEFAULT_UNIT_FLAGS.items()), tuple(extra_flags))).encode())
    return h.hexdigest()[:16]


COMMON_FLAGS = ("-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wno-unused-result")
# machine LICM hoists loop-invariant constants into VGPRs: the flat kernel's
# field parser (123 -> 103 VGPRs without it) and the wave kernel (4 waves/SIMD:
# 128 VGPRs + 10 spilled -> 115, none spilled; the 5-wave instance needs it to
# fit 96 VGPRs)
_NO_LICM = ("-mllvm", "-disable-machine-licm")
DEFAULT_UNIT_FLAGS = {"j2t_kern_flat.hip": _NO_LICM, "j2t_kern_wave.hip": _NO_LICM, "j2t_kern_wave5.hip": _NO_LICM,
                      "t2j_kern.hip": _NO_LICM}  # t2j: 144 -> 105 VGPRs
MARK = b"dgj2t-build:"


def _deps(unit: str):
    """unit + the csrc/include headers it includes, transitively."""
    import re
    seen, todo = [], [unit]
    while todo:
        f = todo.pop()
        if f in seen:
            continue
        seen.append(f)
        p = os.path.join(CSRC, f) if os.path.exists(os.path.join(CSRC, f)) else os.path.join(ROOT, "include", f)
        with open(p) as fh:
            for inc in re.findall(r'^\s*#\s*include\s+"([^"]+)"', fh.read(), re.M):
                todo.append(os.path.basename(inc))
    return sorted(seen)


def unit_hash(unit: str, extra_flags=()) -> str:
    h = hashlib.sha256()
    for f in _deps(unit):
        p = os.path.join(CSRC, f) if os.path.exists(os.path.join(CSRC, f)) else os.path.join(ROOT, "include", f)
        with open(p, "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    h.update(repr((ARCH, COMMON_FLAGS, tuple(extra_flags))).encode())
    return h.hexdigest()[:16]


def embedded_hash(path: str):
    """The source hash compiled into a built library (dg_build_info), read
    from the file without loading it."""
    try:
        with open(path, "rb") as fh:
            data = fh.read()
    except OSError:
        return None
    k = data.find(MARK)
    if k < 0:
        return None
    return data[k + len(MARK):k + len(MARK) + 16].decode("ascii", "replace")


def build_hip(force=False, extra_flags=(), out=None, unit_flags=None):
    """Compile the translation units in parallel (one hipcc each), then link.
    Skipped only when the existing library carries the hash of exactly these
    sources + flags (compiled in as dg_build_info); a library built from
    anything else is rebuilt."""
    out = out or os.path.join(ROOT, "dynamicgo_amd", "libdgj2t.so")
    unit_flags = unit_flags or {}
    sh = source_hash(tuple(extra_flags) + tuple(sorted((u, tuple(f)) for u, f in unit_flags.items())))
    uf0 = dict(DEFAULT_UNIT_FLAGS)
    for u, f in unit_flags.items():
        uf0[u] = tuple(uf0.get(u, ())) + tuple(f)
    unit_flags = uf0
    if not force and embedded_hash(out) == sh:
        print(f"libdgj2t.so up to date (sources {sh})", flush=True)
        return out
    objdir = os.path.join(ROOT, "build", "obj")
    os.makedirs(objdir, exist_ok=True)
    common = [HIPCC, f"--offload-arch={ARCH}", *COMMON_FLAGS, *extra_flags]
    procs, objs = [], []
    for u in UNITS:
        # objects are cached by the hash of what they are built from; the
        # host unit also carries the library hash (dg_build_info)
        uf = tuple(extra_flags) + tuple(unit_flags.get(u, ()))
        uh = unit_hash(u, uf) + (sh if u == "j2t_host.hip" else "")
        o = os.path.join(objdir, u.replace(".hip", "") + "_" + uh + ".o")
        objs.append(o)
        if os.path.exists(o) and not force:
            continue
        cmd = common + list(unit_flags.get(u, ())) + ([f'-DDG_SRC_HASH="{sh}"'] if u == "j2t_host.hip" else [])
        cmd = cmd + ["-c", "-o", o + ".tmp", os.path.join(CSRC, u)]
        print("+", " ".join(cmd), flush=True)
        procs.append((u, o, subprocess.Popen(cmd)))
    failed = [u for u, o, p in procs if p.wait() != 0]
    if failed:
        raise RuntimeError(f"hipcc failed on {failed}")
    for u, o, p in procs:
        os.replace(o + ".tmp", o)
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp", *objs])
    os.replace(out + ".tmp", out)
    if embedded_hash(out) != sh:
        raise RuntimeError("built library does not carry its source hash")
    return out


def build_oracle():
    _run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "oracle"])
    if os.path.isdir("/root/reference/native"):
        _run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"])


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    build_hip(force="--force" in argv)
    if "--no-oracle" not in argv:
        build_oracle()


if __name__ == "__main__":
    main()
