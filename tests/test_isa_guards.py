"""Guards on the compiled gfx950 assembly (CPU: hipcc cross-compiles, nothing runs).

The KKT kernels' LDS-DMA blocks (lqr.jl_amd/csrc/lqrx_stage.h dma_lds) set M0 and do not
restore it.  That is only sound while the compiler itself never uses M0 in the translation
units that issue them.  For every csrc/*.hip that calls dma_lds this test
  * checks the source for constructs whose code generation uses M0 (the LDS-DMA builtins,
    stage_chunk which wraps them, s_sendmsg, GWS, LDS-param / readlane-by-M0 intrinsics), and
  * compiles the file to assembly and fails if any instruction outside the inline-asm
    blocks reads or writes m0.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "lqr.jl_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

# source constructs that make the compiler write M0 (or rely on it across instructions)
M0_USERS = re.compile(r"__builtin_amdgcn_(global_load_lds|raw_buffer_load_lds|raw_ptr_buffer_load_lds|"
                      r"load_to_lds|s_sendmsg\w*|ds_gws\w*|ds_append|ds_consume|interp\w*|lds_param\w*)"
                      r"|\bstage_chunk\s*\(|s_sendmsg|ds_gws")


def _dma_units():
    out = []
    for f in sorted(os.listdir(CSRC)):
        if f.endswith(".hip"):
            src = open(os.path.join(CSRC, f)).read()
            if re.search(r"\bdma_lds\s*<", src):
                out.append(f)
    return out


DMA_UNITS = _dma_units()


def test_dma_units_found():
    assert "lqrx_kkt_fil.hip" in DMA_UNITS, DMA_UNITS


@pytest.mark.parametrize("unit", DMA_UNITS)
def test_dma_unit_source_has_no_m0_users(unit):
    src = open(os.path.join(CSRC, unit)).read()
    # strip comments before scanning
    src = re.sub(r"//[^\n]*", "", re.sub(r"/\*.*?\*/", "", src, flags=re.S))
    hits = sorted(set(m.group(0) for m in M0_USERS.finditer(src)))
    assert not hits, f"{unit} uses M0-writing constructs beside dma_lds: {hits}"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("unit", DMA_UNITS)
def test_dma_unit_leaves_m0_to_the_dma_blocks(unit, tmp_path):
    out = tmp_path / (unit + ".s")
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                    "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S",
                    os.path.join(CSRC, unit), "-o", str(out)], check=True, timeout=900)
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
