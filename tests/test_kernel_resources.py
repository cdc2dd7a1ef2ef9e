"""Kernel resources read from the built libndfl.so (its gfx950 code object's metadata notes), CPU only.

The strict stage (ndfl_inflate_strict_kernel) must not use scratch memory: builds of it that did --
a call to a non-inlined helper (its stack) or register spills -- lost real block headers at full
load, nondeterministically (tests/test_gpu_headers.py compares the accepted
set with the oracle).  The header finder and the count/emit passes are listed with their VGPRs and
spills for the record (profiles/ quote them).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "deflate-library-java_amd", "lib", "libndfl.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def kernel_metadata(lib=LIB, tmp="/tmp"):
    """{kernel name: {key: int}} from the .hip_fatbin's gfx950 code object (llvm-readelf --notes)."""
    fb = os.path.join(tmp, f"ndfl_fatbin_{os.getpid()}.bin")
    co = os.path.join(tmp, f"ndfl_co_{os.getpid()}.o")
    cp = os.path.join(tmp, f"ndfl_lib_{os.getpid()}.so")
    try:
        # (on a copy: objcopy with one file argument rewrites that file, which would corrupt the
        # library a test process already has mapped)
        shutil.copyfile(lib, cp)
        subprocess.check_call(["objcopy", "--dump-section", f".hip_fatbin={fb}", cp, cp + ".out"])
        subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}", f"--output={co}"])
        notes = subprocess.check_output([os.path.join(LLVM, "llvm-readelf"), "--notes", co], text=True)
    finally:
        for f in (fb, co, cp, cp + ".out"):
            if os.path.exists(f):
                os.remove(f)
    kernels, entry = {}, None
    for line in notes.splitlines():
        if re.match(r"\s*- \.", line):                 # a new kernel entry (keys come alphabetically)
            entry = {}
        m = re.match(r"\s*-?\s*\.name:\s+(\S+)$", line)
        if m and entry is not None and not m.group(1).endswith(".kd"):
            kernels[m.group(1)] = entry
            continue
        m = re.match(r"\s*-?\s*\.(private_segment_fixed_size|vgpr_count|vgpr_spill_count|sgpr_spill_count|"
                     r"group_segment_fixed_size):\s+(\d+)$", line)
        if m and entry is not None:
            entry[m.group(1)] = int(m.group(2))
    return kernels


needs_tools = pytest.mark.skipif(not (os.path.exists(LIB) and shutil.which("objcopy") and
                                      os.path.exists(os.path.join(LLVM, "llvm-readelf"))),
                                 reason="needs the built library and the ROCm LLVM tools")


@needs_tools
def test_strict_stage_uses_no_scratch():
    k = kernel_metadata()["ndfl_inflate_strict_kernel"]
    assert k["private_segment_fixed_size"] == 0, k
    assert k["vgpr_spill_count"] == 0, k
    # 5 waves per SIMD: 512 / 5 -> at most 96 VGPRs (granule 8), and 5 workgroups' tables in LDS
    assert k["vgpr_count"] <= 96, k
    assert 5 * k["group_segment_fixed_size"] <= 160 * 1024, k


@needs_tools
def test_every_exported_kernel_has_metadata():
    ks = kernel_metadata()
    for name in ("ndfl_inflate_find_compact_kernel", "ndfl_inflate_count_wave_kernel",
                 "ndfl_inflate_emit_fast_kernel", "ndfl_deflate_hist_kernel", "ndfl_deflate_emit_kernel"):
        assert name in ks and ks[name]["vgpr_count"] > 0, name
