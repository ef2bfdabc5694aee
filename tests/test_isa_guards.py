"""Guards on the compiled gfx950 assembly (CPU: hipcc cross-compiles, nothing runs).

The KKT kernel's LDS-DMA blocks (lqr.jl_amd/csrc/lqrx_stage.h dma_lds) set M0 and do not
restore it.  That is only sound while the compiler itself never uses M0 in the kernels that
include them: this test compiles lqrx_kkt_fil.hip to assembly and fails if any instruction
outside the inline-asm blocks reads or writes m0.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "lqr.jl_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_fil_kernel_leaves_m0_to_the_dma_blocks(tmp_path):
    out = tmp_path / "fil.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                    "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S",
                    os.path.join(CSRC, "lqrx_kkt_fil.hip"), "-o", str(out)], check=True, timeout=600)
    inasm, bad, dma = False, [], 0
    for line in out.read_text().splitlines():
        t = line.strip()
        if t.startswith(";;#ASMSTART"):
            inasm = True
            continue
        if t.startswith(";;#ASMEND"):
            inasm = False
            continue
        if inasm:
            dma += "lds" in t and t.startswith("buffer_load")
            continue
        if t and not t.startswith((";", ".")) and "m0" in t.replace(",", " ").split():
            bad.append(t)
    assert dma > 0, "no LDS-DMA blocks found (kernel changed?)"
    assert not bad, f"compiler uses M0 outside the DMA blocks: {bad[:5]}"
