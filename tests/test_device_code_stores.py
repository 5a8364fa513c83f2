"""Device code writes memory through vector stores only: no scalar-cache stores, scalar atomics or
scalar-cache write-backs anywhere in libmxp's gfx950 code objects (this pool forbids them).  CPU test:
disassembles the built objects.  (Listed in .gpurunignore: no GPU run needs it.)"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
OBJS = ["kernels.hip.o", "resolve.hip.o", "lists.hip.o", "quota.hip.o", "pack.hip.o"]
FORBIDDEN = re.compile(r"^\s+s_(store|atomic|buffer_store|buffer_atomic|dcache_wb|dcache_discard|scratch_store)\w*",
                       re.M)


@pytest.mark.parametrize("obj", OBJS)
def test_no_scalar_memory_writes(tmp_path, obj):
    from istio_amd import build
    build.build()
    src = os.path.join(ROOT, "istio_amd", "build", obj)
    fat = tmp_path / "fat.bin"
    co = tmp_path / "k.co"
    subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=%s" % fat, src, os.devnull])
    subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=%s" % fat,
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=%s" % co])
    asm = subprocess.check_output([os.path.join(LLVM, "llvm-objdump"), "-d", str(co)]).decode()
    assert "global_store" in asm or "global_atomic" in asm or "buffer_store" in asm
    bad = FORBIDDEN.findall(asm)
    assert not bad, bad[:5]
