"""Per-iteration schedule summary of a loop in gfx950 assembly: issued instructions by class and
the longest register dependency chain through one iteration (RAW edges only, unit weight, and
weighted by a rough per-class latency) — critical-path length against issued instructions.

    python tools/chain_len.py ASM.s FUNCTION_SUBSTRING [--loop N]

ASM.s: `hipcc --cuda-device-only -S` output.  The loops are the backward branches of the
function (target label before the branch); --loop picks one (default: the first).  The model is
deliberately simple: the first operand of a VALU/SALU/DS-load/VMEM-load instruction is its
destination, the others its sources (stores have no destination); v_readlane's destination is an
SGPR; vcc/exec dependencies are ignored.  Latencies: fp64 VALU 8, other VALU 4, DPP move 8,
transcendental 16, DS read 64, VMEM load 500 (issue-to-use), SALU 1, readlane 8.
"""
import re
import sys
from collections import Counter

LAT = [(re.compile(r"^v_(rsq|rcp|sqrt|exp|log)_"), 16), (re.compile(r"^v_\w+_f64"), 8),
       (re.compile(r"^v_mov_b32_dpp|_dpp$"), 8), (re.compile(r"^v_readlane"), 8), (re.compile(r"^v_"), 4),
       (re.compile(r"^ds_(read|bpermute)"), 64), (re.compile(r"^(global|buffer|flat|scratch)_load"), 500),
       (re.compile(r"^s_"), 1)]
REG = re.compile(r"\b([vs])(\d+)\b|\b([vs])\[(\d+):(\d+)\]")


def regs(txt):
    out = []
    for m in REG.finditer(txt):
        if m.group(1):
            out.append((m.group(1), int(m.group(2))))
        else:
            out += [(m.group(3), r) for r in range(int(m.group(4)), int(m.group(5)) + 1)]
    return out


def lat(op):
    for rx, v in LAT:
        if rx.search(op):
            return v
    return 1


def main():
    path, fn = sys.argv[1], sys.argv[2]
    which = int(sys.argv[sys.argv.index("--loop") + 1]) if "--loop" in sys.argv else 0
    s = open(path).read()
    name = next(n for n in re.findall(r"^(_Z\w+):", s, re.M) if fn in n)
    body = s[s.find(name + ":"):s.find(".Lfunc_end", s.find(name + ":"))].split("\n")
    labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\d+_\d+):", l.strip()))}
    loops = [(labels[m.group(1)], i) for i, l in enumerate(body)
             if (m := re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)", l)) and m.group(1) in labels
             and labels[m.group(1)] < i]
    a, b = loops[which]
    cls, last, depth, wdepth = Counter(), {}, {}, {}
    crit = wcrit = n = 0
    for l in body[a:b + 1]:
        t = l.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        op, _, rest = t.partition(" ")
        n += 1
        cls["mfma" if "mfma" in op else "valu" if op.startswith("v_") else "salu" if op.startswith("s_")
            else "lds" if op.startswith("ds_") else "vmem"] += 1
        ops = [x.strip() for x in rest.split(",")]
        store = re.match(r"^(ds_write|global_store|buffer_store|scratch_store|flat_store)", op)
        dst = [] if (store or op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_cbranch", "s_branch"))) \
            else regs(ops[0]) if ops and ops[0] else []
        src = regs(",".join(ops if not dst else ops[1:]))
        d0 = max([depth.get(r, 0) for r in src] + [0]) + 1
        w0 = max([wdepth.get(r, 0) for r in src] + [0]) + lat(op)
        for r in dst:
            depth[r], wdepth[r] = d0, w0
        crit, wcrit = max(crit, d0), max(wcrit, w0)
    print(f"{name} loop {which} (lines {a}-{b}): {n} instructions {dict(cls)}; "
          f"longest RAW chain {crit} instructions, ~{wcrit} cycles by the latency model")


if __name__ == "__main__":
    main()
