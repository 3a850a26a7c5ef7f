"""CPU check of the built library's gfx950 code object: the solve kernels keep
their working set in registers and LDS.  A kernel with private (scratch)
memory in its Dijkstra loop pays a scratch round trip per step -- round 3's
register-tile kernel had its tile in 384 B of scratch while two solvers were
inlined into one instantiation (santa_vt_kernel, now one solver each).

Reads the AMDGPU metadata notes of the code object bundled in
libsanta_hip.so (llvm-objcopy + clang-offload-bundler + llvm-readelf from
/opt/rocm); skipped when the library or the tools are absent."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(ROOT, "mpi-hungarian-method_amd", "santa_hip", "libsanta_hip.so")

# kernels that run in a default round or a test of the product path (the
# TIMED / A-B instantiations and the int16 tile build's one-time prologue
# spill -- santa_tile_kernel<0>, 28 dwords, outside its loops -- are not
# held to it)
NO_SCRATCH = (
    "santa_tile_kernelILi1E",
    "santa_sp3_kernelILb0ELb0E", "santa_sp3_kernelILb0ELb1E", "santa_dt_kernel", "santa_vt_kernelILi0ELi1E", "santa_vt_kernelILi0ELi0E",
    "santa_block_kernelILi1ELi0ELb0E", "santa_block_kernelILi1ELi1ELb0E",
    "santa_big_kernel", "santa_lb_kernel", "score_kernel", "lsap_i64_kernel", "lsap_f64_kernel",
)


def _kernel_meta(tmp_path):
    tools = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf")]
    if not os.path.exists(LIB) or not all(os.path.exists(t) for t in tools):
        pytest.skip("library or ROCm LLVM tools absent")
    objcopy, bundler, readelf = tools
    fb, co = str(tmp_path / "fb.bin"), str(tmp_path / "co.o")
    subprocess.run([objcopy, f"--dump-section=.hip_fatbin={fb}", LIB, str(tmp_path / "junk.so")], check=True)
    subprocess.run([bundler, "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}",
                    f"--output={co}", "--unbundle"], check=True)
    notes = subprocess.run([readelf, "--notes", co], check=True, capture_output=True, text=True).stdout
    meta = {}
    for block in re.split(r"\n\s+- \.", notes):
        name = re.search(r"\.?name:\s+(_Z\S+)", block)
        priv = re.search(r"\.private_segment_fixed_size:\s+(\d+)", block)
        if name and priv:
            meta[name.group(1)] = int(priv.group(1))
    return meta


def test_solve_kernels_use_no_scratch(tmp_path):
    meta = _kernel_meta(tmp_path)
    assert meta, "no kernel metadata found in the code object"
    checked = {k: v for k, v in meta.items() if any(p in k for p in NO_SCRATCH)}
    for p in NO_SCRATCH:
        assert any(p in k for k in checked), f"kernel {p} missing from the code object"
    bad = {k: v for k, v in checked.items() if v}
    assert not bad, f"kernels with private (scratch) memory: {bad}"
