"""Build libmxp.so (host C++ + gfx950 HIP kernels) in-tree with hipcc.

    python -m istio_amd.build          # or istio_amd.build.build()

The shared library is the engine's C-ABI (include/mxp.h); it is what a cgo shim or the ctypes
host mirror (istio_amd/engine.py) loads.  Built for gfx950 (MI355X) only.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libmxp.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("MXP_OFFLOAD_ARCH", "gfx950")

SOURCES = ["goutil.cpp", "frontend.cpp", "ilgen.cpp", "lower.cpp", "vmopt.cpp", "regex.cpp", "engine.cpp",
           "resolver.cpp", "refs.cpp", "wire.cpp", "lists.cpp", "quota.cpp", "pack_device.cpp", "kernels.hip", "resolve.hip", "lists.hip", "quota.hip", "pack.hip", "group.cpp", "group.hip"]
HEADERS = ["goutil.h", "frontend.h", "ilgen.h", "lower.h", "vmopt.h", "vm.h", "kargs.h", "engine_impl.h", "resolve_args.h", "netparse.h", "timeparse.h", "lists.h", "regex.h", "unicode_tables.h", "dfa_dev.h", "quota_args.h", "pack_args.h", "par.h", "goupper.h", "upper_table.h"]


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps += [os.path.join(HERE, "..", "include", f) for f in ("mxp.h", "mxp_batch.h", "mxp_group.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    # MXP_NO_BUILD=1 (GPU session scripts): use the library as shipped, whatever the sources' times
    if not force and os.environ.get("MXP_NO_BUILD") == "1" and os.path.exists(LIB):
        return LIB
    if not force and not _stale():
        return LIB
    # one builder at a time (the ranks of a multi-GPU bench all call build()): the others wait on
    # the lock and then find the library up to date
    import fcntl
    with open(LIB + ".lock", "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        if not force and not _stale():
            return LIB
        return _build(verbose)


def _build(verbose: bool) -> str:
    objdir = os.path.join(HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    objs = []
    procs = []
    for src in SOURCES:
        obj = os.path.join(objdir, src + ".o")
        objs.append(obj)
        cmd = [HIPCC, "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
               "--offload-arch=" + ARCH, "-c", os.path.join(CSRC, src), "-o", obj]
        if not src.endswith(".hip"):
            cmd.insert(1, "-x")
            cmd.insert(2, "hip")
        if verbose:
            print(" ".join(cmd))
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    failed = []
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed.append((src, out.decode(errors="replace")))
        elif verbose and out:
            print(out.decode(errors="replace"))
    if failed:
        msg = "\n".join("== %s\n%s" % f for f in failed)
        raise RuntimeError("libmxp build failed:\n" + msg)
    tmp = LIB + ".tmp"
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs + ["-ldl"]
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
