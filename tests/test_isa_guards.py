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


@pytest.fixture(scope="module")
def asm_of(tmp_path_factory):
    """gfx950 assembly of every unit these guards read, compiled once and concurrently (each
    unit is a multi-minute hipcc run; the CPU suite runs serially)."""
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    d = tmp_path_factory.mktemp("isa")
    units = sorted(set(DMA_UNITS) | {"lqrx_dp.hip"})
    procs = {}
    for u in units:
        procs[u] = subprocess.Popen([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                                     "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S",
                                     os.path.join(CSRC, u), "-o", str(d / (u + ".s"))],
                                    stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    for u, pr in procs.items():
        assert pr.wait(timeout=1200) == 0, f"hipcc failed on {u}"
    return lambda u: (d / (u + ".s")).read_text()


def test_dma_units_found():
    assert "lqrx_kkt_fil.hip" in DMA_UNITS, DMA_UNITS


@pytest.mark.parametrize("unit", DMA_UNITS)
def test_dma_unit_source_has_no_m0_users(unit):
    src = open(os.path.join(CSRC, unit)).read()
    # strip comments before scanning
    src = re.sub(r"//[^\n]*", "", re.sub(r"/\*.*?\*/", "", src, flags=re.S))
    hits = sorted(set(m.group(0) for m in M0_USERS.finditer(src)))
    assert not hits, f"{unit} uses M0-writing constructs beside dma_lds: {hits}"


@pytest.mark.parametrize("unit", DMA_UNITS)
def test_dma_unit_leaves_m0_to_the_dma_blocks(unit, asm_of):
    inasm, bad, dma = False, [], 0
    for line in asm_of(unit).splitlines():
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


def _regs(text):
    out = set()
    for a, b in re.findall(r"v\[(\d+):(\d+)\]", text):
        out.update(range(int(a), int(b) + 1))
    for a in re.findall(r"\bv(\d+)\b", re.sub(r"v\[\d+:\d+\]", "", text)):
        out.add(int(a))
    return out


def test_dp_rollout_asm_loads_not_read_before_their_wait(asm_of):
    """The DP rollout (lqrx_dp.hip dp_rollout_full) issues its K loads as inline asm, invisible
    to the compiler's wait-count pass, and waits for them by hand.  The compiler treats an asm
    output register as written at the asm statement, so it may copy it (or read it otherwise)
    before the hand wait — a race it cannot see: round 4 found one in the linear-terms variant
    (an in-flight d_k register copied before the wait; intermittently wrong X/U).  Guard: in the
    compiled gfx950 assembly of every dp_riccati_kernel, no instruction outside the inline-asm
    blocks reads a register an inline-asm load wrote before an s_waitcnt vmcnt follows it."""
    text = asm_of("lqrx_dp.hip")
    bad, kernels, asm_loads = [], 0, 0
    for m in re.finditer(r"^(_ZN4lqrx17dp_riccati_kernel\w+):", text, re.M):
        kernels += 1
        body = text[m.end():text.find(".Lfunc_end", m.end())]
        inasm, pend = False, {}
        for ln in body.split("\n"):
            s = ln.strip()
            if s.startswith(";;#ASMSTART"):
                inasm = True
                continue
            if s.startswith(";;#ASMEND"):
                inasm = False
                continue
            if not s or s.startswith(";") or s.startswith("."):
                continue
            if "s_waitcnt" in s and "vmcnt" in s:
                pend = {}
                continue
            if inasm:
                lm = re.match(r"global_load_dword\w*\s+(v\[\d+:\d+\]|v\d+)", s)
                if lm:
                    asm_loads += 1
                    for r in _regs(lm.group(1)):
                        pend[r] = s
                continue
            if s.startswith("s_"):
                continue
            hit = _regs(s) & set(pend)
            if hit:
                bad.append((m.group(1)[-48:], s, pend[min(hit)]))
    assert kernels > 0 and asm_loads > 0, (kernels, asm_loads)
    assert not bad, bad[:5]
