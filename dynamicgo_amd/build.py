"""Build the in-tree native artefacts.

  dynamicgo_amd/libdgj2t.so        HIP kernels + C ABI for gfx950 (the product)
  oracle/_build/libj2t_oracle.so   plain-C restatement (test infrastructure)
  oracle/_ref/libdgref*.so         the reference's own native/*.c (test
                                   infrastructure; only when /root/reference exists)

Usage: python -m dynamicgo_amd.build [--no-oracle]
"""
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


UNITS = ("j2t_kern_wave.hip", "j2t_kern_small.hip", "j2t_kern_lds.hip", "j2t_kern_glb.hip", "j2t_host.hip")
HEADERS = ("j2t_small.h", "j2t_wave.h", "j2t_machine.h", "j2t_device.h", "j2t_fast.h", "dg_tables.h")


def build_hip(force=False, extra_flags=(), out=None):
    """Compile the translation units in parallel (one hipcc each), then link."""
    out = out or os.path.join(ROOT, "dynamicgo_amd", "libdgj2t.so")
    srcs = [os.path.join(CSRC, f) for f in UNITS + HEADERS]
    srcs += [os.path.join(ROOT, "include", f) for f in ("dgj2t.h", "dgj2t_desc.h")]
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(s) for s in srcs):
        return out
    objdir = os.path.join(ROOT, "build", "obj" + ("_" + str(abs(hash(tuple(extra_flags)))) if extra_flags else ""))
    os.makedirs(objdir, exist_ok=True)
    common = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
              "-Wno-unused-result", *extra_flags]
    procs, objs = [], []
    for u in UNITS:
        o = os.path.join(objdir, u.replace(".hip", ".o"))
        cmd = common + ["-c", "-o", o, os.path.join(CSRC, u)]
        print("+", " ".join(cmd), flush=True)
        procs.append((u, subprocess.Popen(cmd)))
        objs.append(o)
    failed = [u for u, p in procs if p.wait() != 0]
    if failed:
        raise RuntimeError(f"hipcc failed on {failed}")
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out, *objs])
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
