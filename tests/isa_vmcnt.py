"""Static model of `s_waitcnt vmcnt(N)` over compiled gfx950 assembly (test infrastructure only).

Some kernels issue loads the compiler's wait-count pass cannot see and wait for them by hand:
  * the DP rollout's K loads (lqrx_dp.hip dp_rollout_full: inline-asm `global_load_dword*` into
    a register ring, waited by `vm_wait_regs<VMW>`), and
  * the KKT kernels' LDS-DMA staging (lqrx_kkt_fil.hip `dma_lds`, inline-asm
    `buffer_load_* … lds`; lqrx_kkt.hip `stage_chunk`, `global_load_lds_*`), waited by
    `vm_wait<N, G>` / `dma_wait_but<N>`.
A bound N that is too lax lets a consumer run before its data has landed — an intermittent wrong
answer (round 4 shipped one: the compiler copied an in-flight asm-loaded register before the
hand wait).  This module checks the bounds against the instruction stream that was actually
compiled.

Hardware model (the one the compiler's own SIInsertWaitcnts pass uses for gfx9/CDNA, where loads
and stores share one counter): every vector-memory instruction (MUBUF/MTBUF/FLAT/GLOBAL/SCRATCH
load, store, atomic, LDS-DMA) increments vmcnt when issued, and they retire IN ISSUE ORDER;
`s_waitcnt vmcnt(N)` returns once at most N are outstanding, i.e. every op except the N most
recently issued has completed.  So an op is complete after a `vmcnt(N)` iff at least N VMEM
instructions were issued after it.  (Cache-control ops — buffer_wbl2 / buffer_inv — are not
counted: undercounting the ops issued after a load only makes the check stricter.)

Analysis: a forward dataflow over the function's control-flow graph (basic blocks split at
labels and branches, loops iterated to a fixed point).  State:
  * pending registers: for every VGPR that is the destination of an inline-asm load not yet
    known complete, the MINIMUM over paths of the number of VMEM instructions issued since;
  * DMA groups (source-marked: `; lqrx.grp` opens a group, inline asm of the staging code): the
    most recent groups, each with the minimum number of VMEM instructions issued after its last
    DMA instruction (∞ before its first DMA, or once a wait has retired it).
A join takes the union of pending registers and the position-wise minimum (newest aligned) of
the groups — sound for every real path (the real path's count is one of the minimised ones);
infeasible paths can only add false alarms.
Findings:
  * `hazard`: an instruction outside the inline-asm blocks names (reads or overwrites) a
    pending register — the compiler moved or copied a value whose load may not have landed, or
    reused the register while a late load can still overwrite it;
  * `bound`: a tagged hand wait `s_waitcnt vmcnt(N) … ; lqrx.wait g=G` whose target — the G-th
    most recent DMA group — has fewer than N VMEM instructions after its last DMA on some path;
  * `untagged`: a hand wait with N > 0 inside inline asm that names no target group, in a
    function that issues DMA (an unchecked bound).
"""
import functools
import re

INF = 1 << 30
CAP = 64               # vmcnt is 6 bits on gfx9: counts past 63 all mean "retired by any wait"
MAXG = 8               # DMA groups remembered

VMEM = re.compile(r"^(global|buffer|flat|scratch|tbuffer)_(load|store|atomic)\w*")
WAIT = re.compile(r"^s_waitcnt\b(.*)")
BRANCH = re.compile(r"^s_(branch|cbranch_\w+)\s+(\S+)")
LABEL = re.compile(r"^([.\w$]+):")
TAG = re.compile(r"lqrx\.wait\s+g=(\d+)")


@functools.lru_cache(maxsize=None)
def regs(text):
    """VGPR numbers named in an operand string (v7, v[4:7]) (memoised: the dataflow revisits the
    same instruction text many times)."""
    out = set()
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", text):
        out.update(range(int(a), int(b) + 1))
    for a in re.findall(r"\bv(\d+)\b", re.sub(r"\bv\[\d+:\d+\]", "", text)):
        out.add(int(a))
    return frozenset(out)


def vmcnt_of(wait_operands):
    """N of a `s_waitcnt` operand string, or None when it does not wait on vmcnt."""
    s = wait_operands.split(";")[0].strip()
    m = re.search(r"vmcnt\((\d+)\)", s)
    if m:
        return int(m.group(1))
    if re.fullmatch(r"0|0x0", s):
        return 0
    return None


def functions(asm, name_re):
    """{symbol: [(text, inasm, lineno)]} for every function whose symbol matches name_re."""
    out = {}
    lines = asm.split("\n")
    for m in re.finditer(r"^(" + name_re + r"):[ \t]*(?:;.*)?$", asm, re.M):
        sym = m.group(1)
        start = asm.count("\n", 0, m.end()) + 1
        body, inasm = [], False
        for i in range(start, len(lines)):
            s = lines[i].strip()
            if s.startswith(".Lfunc_end"):
                break
            if s.startswith(";;#ASMSTART"):
                inasm = True
                continue
            if s.startswith(";;#ASMEND"):
                inasm = False
                continue
            if not s:
                continue
            if LABEL.match(s) and not inasm:
                body.append((s, False, i + 1))
                continue
            if s.startswith(";"):
                if inasm and "lqrx." in s:
                    body.append((s, True, i + 1))          # a source marker
                continue
            if s.startswith("."):
                continue
            body.append((s, inasm, i + 1))
        out[sym] = body
    return out


def blocks(body):
    """Basic blocks [label, [instrs], [successor labels], condition] in layout order; a conditional
    branch's successors are [taken, fall-through] and its condition the branch mnemonic's tail
    (cbranch_vccnz, cbranch_scc0, …)."""
    bl, cur, lab, n = [], [], "<entry>", 0

    def close(succ, cond=None):
        nonlocal cur, lab, n
        bl.append([lab, cur, succ, cond])
        n += 1
        cur, lab = [], f"<fall{n}>"

    for ins in body:
        s, inasm, _ = ins
        m = LABEL.match(s)
        if m and not inasm:
            if cur or lab.startswith("<fall"):
                close(None)                                # falls through into the label
            lab = m.group(1)
            continue
        cur.append(ins)
        if inasm:
            continue
        b = BRANCH.match(s)
        if b:
            close([b.group(2)] if b.group(1) == "branch" else [b.group(2), None],
                  None if b.group(1) == "branch" else b.group(1))
        elif s.startswith(("s_endpgm", "s_setpc_b64", "s_trap")):
            close([])
    if cur:
        close([])
    # resolve fall-through successors (None) to the next block's label
    for i, b in enumerate(bl):
        if b[2] is None:
            b[2] = [bl[i + 1][0]] if i + 1 < len(bl) else []
        else:
            b[2] = [s if s is not None else (bl[i + 1][0] if i + 1 < len(bl) else None) for s in b[2]]
            if None in b[2]:
                b[2], b[3] = [s for s in b[2] if s is not None], None
    return bl


def _join_state(a, b):
    if a is None:
        return b
    pa, ga = a
    pb, gb = b
    p = dict(pa)
    for r, c in pb.items():
        p[r] = min(c, p.get(r, INF))
    n = max(len(ga), len(gb))
    g = []
    for i in range(n):          # position from the oldest of the aligned (newest-last) tails
        x = ga[i - n + len(ga)] if i - n + len(ga) >= 0 else INF
        y = gb[i - n + len(gb)] if i - n + len(gb) >= 0 else INF
        g.append(min(x, y))
    return (p, tuple(g[-MAXG:]))


def _join(a, b):
    """Disjunctive join: states are kept apart per branch-flag signature (see _flags)."""
    if a is None:
        return dict(b)
    out = dict(a)
    for sig, st in b.items():
        out[sig] = _join_state(out.get(sig), st)
    return out


@functools.lru_cache(maxsize=None)
def sregs(text):
    """SGPR numbers named in an operand string (s7, s[4:5])."""
    out = set()
    for a, b in re.findall(r"\bs\[(\d+):(\d+)\]", text):
        out.update(range(int(a), int(b) + 1))
    for a in re.findall(r"\bs(\d+)\b", re.sub(r"\bs\[\d+:\d+\]", "", text)):
        out.add(int(a))
    return frozenset(out)


VCCDEF = re.compile(r"^s_(and|andn2)_b64\s+vcc,\s*exec,\s*(s\[\d+:\d+\])\s*$")


def _flag_regs(body):
    """SGPR pairs the compiler uses as branch flags: `s_and[n2]_b64 vcc, exec, s[a:b]` followed by
    a vcc branch.  Their constant values (`s_mov_b64 s[a:b], 0 / -1`) are tracked per path, so a
    diamond laid out as two sequential tests of one flag is not read as a path through neither
    (or both) of its arms."""
    out = set()
    for s, inasm, _ in body:
        m = VCCDEF.match(s.split(";")[0].strip())
        if m:
            out.add(m.group(2))
    return out


@functools.lru_cache(maxsize=None)
def _sig_update(sig, s, flags):
    """New flag signature after instruction s (sig: tuple of (flag, value) incl. ('vcc', bool))."""
    d = dict(sig)
    t = s.split(";")[0].strip()
    mnem, _, ops = t.partition(" ")
    opl = [o.strip() for o in ops.split(",")] if ops else []
    m = VCCDEF.match(t)
    if m:
        v = d.get(m.group(2))
        if v is None:
            d.pop("vcc", None)
        elif m.group(1) == "andn2":
            d["vcc"] = {-1: False, 0: True}.get(v)
        else:
            d["vcc"] = {-1: True, 0: False}.get(v)
        if d.get("vcc") is None:
            d.pop("vcc", None)
        return tuple(sorted(d.items(), key=str))
    if not opl or mnem.startswith(("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_nop",
                                   "s_setprio", "s_barrier", "s_endpgm", "s_sleep")):
        return sig
    dst = opl[0]
    if "vcc" in dst.split() or dst == "vcc":
        d.pop("vcc", None)
    if mnem.startswith(("v_cmp", "v_cmpx")) and (mnem.endswith("_e32")):
        d.pop("vcc", None)                          # e32 compares write vcc implicitly
    ds = sregs(dst) if not mnem.startswith(("global_", "buffer_", "flat_", "scratch_", "ds_")) else set()
    for f in flags:
        if ds & sregs(f):
            if mnem == "s_mov_b64" and dst == f and re.fullmatch(r"-?\d+", opl[1] if len(opl) > 1 else ""):
                d[f] = int(opl[1])
            else:
                d.pop(f, None)
    return tuple(sorted(d.items(), key=str))


def _bump(c):
    return c if c >= INF else min(c + 1, CAP)


def _step(state, ins, findings, sym, record):
    pend, groups = dict(state[0]), list(state[1])
    s, inasm, ln = ins
    if s.startswith(";"):                                   # source marker
        if "lqrx.grp" in s:
            groups.append(INF)
            groups = groups[-MAXG:]
        return pend, tuple(groups)
    w = WAIT.match(s)
    if w:
        n = vmcnt_of(w.group(1))
        if n is None:
            return pend, tuple(groups)
        t = TAG.search(s)
        if record:
            if t:
                g = int(t.group(1))
                have = groups[-g] if len(groups) >= g else INF
                if have < n:
                    findings.append(("bound", sym, ln, s, f"target group g={g} has {have} VMEM ops after "
                                                         f"its last DMA on some path, the wait allows {n}"))
            elif inasm and n > 0 and record == "dma":
                findings.append(("untagged", sym, ln, s, "hand vmcnt bound with no target group"))
        pend = {r: c for r, c in pend.items() if c < n}
        groups = [INF if c >= n else c for c in groups]
        return pend, tuple(groups)
    v = VMEM.match(s)
    if v:
        mnem, _, ops = s.partition(" ")
        pend = {r: _bump(c) for r, c in pend.items()}
        groups = [_bump(c) for c in groups]
        dma = " lds" in " " + ops.split(";")[0].replace(",", " ") + " " or "load_lds" in mnem
        if dma:
            if groups:
                groups[-1] = 0
            return pend, tuple(groups)
        opl = [o.strip() for o in ops.split(";")[0].split(",")]
        if inasm:
            if v.group(2) == "load":
                for r in regs(opl[0]):
                    pend[r] = 0
            return pend, tuple(groups)
        # a compiler-issued op: its address / data operands must not be pending; a load's own
        # destination lands after the pending load (in-order) and the compiler waits for it
        rd = regs(",".join(opl[1:])) if v.group(2) == "load" else regs(",".join(opl))
        hit = rd & set(pend)
        if hit and record:
            findings.append(("hazard", sym, ln, s, f"reads in-flight v{min(hit)}"))
        if v.group(2) == "load":
            for r in regs(opl[0]):
                pend.pop(r, None)
        return pend, tuple(groups)
    if inasm or s.startswith("s_"):
        return pend, tuple(groups)
    hit = regs(s.split(";")[0]) & set(pend)
    if hit and record:
        findings.append(("hazard", sym, ln, s, f"names in-flight v{min(hit)}"))
    return pend, tuple(groups)


def _block(bl_i, insig, flags, findings, sym, mode):
    """Transfer one block: {sig: state} in → [(successor label, sig, state)] out."""
    lab, instrs, succ, cond = bl_i
    out = []
    for sig, state in insig.items():
        for x in instrs:
            state = _step(state, x, findings, sym, mode)
            if not x[1]:
                sig = _sig_update(sig, x[0], flags)
        vcc = dict(sig).get("vcc")
        if cond in ("cbranch_vccnz", "cbranch_vccz") and vcc is not None and len(succ) == 2:
            taken = vcc if cond == "cbranch_vccnz" else not vcc
            out.append((succ[0] if taken else succ[1], sig, state))
        else:
            out.extend((t, sig, state) for t in succ)
    return out


def analyse(asm, name_re):
    """Run the model over every function matching name_re.  Returns (findings, stats) with
    stats[sym] = {"asm_loads", "dma", "tagged_waits", "hand_waits"}."""
    findings, stats = [], {}
    for sym, body in functions(asm, name_re).items():
        st = {"asm_loads": 0, "dma": 0, "tagged_waits": 0, "hand_waits": 0}
        for s, inasm, _ in body:
            v = VMEM.match(s)
            if v and (" lds" in s.split(";")[0].replace(",", " ") or "load_lds" in s):
                st["dma"] += 1
            elif v and inasm and v.group(2) == "load":
                st["asm_loads"] += 1
            w = WAIT.match(s)
            if w and inasm and (vmcnt_of(w.group(1)) or 0) > 0:
                st["hand_waits"] += 1
                st["tagged_waits"] += bool(TAG.search(s))
        stats[sym] = st
        if not st["asm_loads"] and not st["dma"]:
            # nothing for the model to find: no inline-asm load can be pending (no hazard), and
            # bound / untagged findings need DMA groups — skip the dataflow (most functions)
            continue
        flags = frozenset(_flag_regs(body))
        bl = blocks(body)
        idx = {b[0]: i for i, b in enumerate(bl)}
        ins = [None] * len(bl)
        ins[0] = {(): ({}, ())}
        work = [0]
        while work:
            i = work.pop(0)
            for t, sig, state in _block(bl[i], ins[i], flags, None, sym, False):
                j = idx.get(t)
                if j is None:
                    continue
                nj = _join(ins[j], {sig: state})
                if nj != ins[j]:
                    ins[j] = nj
                    if j not in work:
                        work.append(j)
        mode = "dma" if st["dma"] else "regs"
        seen = set()
        for i, b in enumerate(bl):
            if ins[i] is not None:                          # (None: unreachable)
                _block(b, ins[i], flags, findings, sym, mode)
        # one finding per instruction (several flag signatures may reach it)
        uniq = []
        for f in findings:
            k = (f[0], f[1], f[2])
            if k not in seen:
                seen.add(k)
                uniq.append(f)
        findings[:] = uniq
    return findings, stats
