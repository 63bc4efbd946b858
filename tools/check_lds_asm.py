"""Check a gfx950 ISA listing for reads of LDS-load destinations before their
s_waitcnt (the wide flush issues ds_read_b64 / ds_read_b128 in
inline asm and waits with a hand-placed lgkmcnt, so the compiler cannot see
those loads; a register copy or spill of a destination between the issue and
the wait would read stale data).

A dataflow pass over each function's control-flow graph: the state is the
ordered list of LGKM operations in flight (each LDS load with its destination
VGPRs; LDS writes and scalar loads as anonymous entries).  `s_waitcnt
lgkmcnt(N)` retires all but the last N.  Any instruction that names a VGPR of
a load still in flight is reported.  At a join the states are merged from the
end (the wait semantics), taking the union of the registers.  Conservative:
scalar loads are counted as in-order LGKM entries.

usage: python tools/check_lds_asm.py volsync_amd/lib/obj/rsync_walk-hip-amdgcn-amd-amdhsa-gfx950.s
(`make -C volsync_amd/csrc asm` writes the listing); exit 1 on a violation.
"""
import re
import sys

BRANCH = re.compile(r"^\s*(s_branch|s_cbranch_\w+)\s+(\S+)")
LABEL = re.compile(r"^([.\w$]+):")
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
WAIT = re.compile(r"lgkmcnt\((\d+)\)")


def regs(text):
    out = set()
    for a, b, c in VREG.findall(text):
        if c:
            out.add(int(c))
        else:
            out.update(range(int(a), int(b) + 1))
    return out


def functions(lines):
    """(name, [(lineno, text)]) for each function body (label .. s_endpgm / .Lfunc_end)."""
    cur, body = None, []
    for i, l in enumerate(lines, 1):
        m = LABEL.match(l)
        if m and not m.group(1).startswith(".") and "@" in l:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
            continue
        if cur is None:
            continue
        if l.startswith(".Lfunc_end"):
            yield cur, body
            cur, body = None, []
            continue
        s = l.split(";")[0].rstrip()
        if s.strip():
            body.append((i, s))
    if cur:
        yield cur, body


def blocks(body):
    """basic blocks: (label, [(lineno, instr)], successor labels)"""
    out, lab, ins = [], "__entry", []
    auto = 0

    def close(succ):
        out.append([lab, ins, succ])

    for ln, s in body:
        m = LABEL.match(s.strip())
        if m:
            close(["@next"])
            lab, ins = m.group(1), []
            continue
        if s.strip().startswith("."):
            continue
        ins.append((ln, s.strip()))
        b = BRANCH.match(s)
        op = s.split()[0]
        if b or op in ("s_endpgm", "s_setpc_b64", "s_trap"):
            succ = []
            if b:
                succ.append(b.group(2))
            if b is None or b.group(1) != "s_branch":
                if op not in ("s_endpgm", "s_setpc_b64"):
                    succ.append("@next")
            close(succ)
            auto += 1
            lab, ins = f"__fall{auto}", []
    close([])
    # resolve "@next"
    for k, blk in enumerate(out):
        blk[2] = [(out[k + 1][0] if t == "@next" and k + 1 < len(out) else t) for t in blk[2]
                  if t != "@next" or k + 1 < len(out)]
    return out


def merge(a, b):
    if a is None:
        return b
    n = max(len(a), len(b))
    pa = [frozenset()] * (n - len(a)) + list(a)
    pb = [frozenset()] * (n - len(b)) + list(b)
    return tuple(x | y for x, y in zip(pa, pb))


CAP = 20   # entries kept apart; older ones are folded into the first (a wait
           # keeps at most the last 15, so they retire together anyway)
_parsed = {}


def parse(s):
    p = _parsed.get(s)
    if p is None:
        op = s.split()[0]
        wait = None
        if op == "s_waitcnt":
            m = WAIT.search(s)
            wait = int(m.group(1)) if m else -1
        kind, dst = None, frozenset()
        if op.startswith("ds_read") or op.startswith("ds_load"):
            kind, dst = "load", frozenset(regs(s.split(None, 1)[1].split(",")[0]))
        elif op.startswith("ds_") or op.startswith("s_load") or op.startswith("s_buffer_load"):
            kind = "other"
        p = _parsed[s] = (op, wait, frozenset(regs(s)), kind, dst)
    return p


def step(state, s, report):
    op, wait, named, kind, dst = parse(s)
    if wait is not None:
        if wait >= 0 and wait < len(state):
            state = state[len(state) - wait:] if wait else ()
        return state
    if state and named:
        for e in state:
            if e & named:
                report(sorted(set().union(*state) & named))
                break
    if kind == "load":
        state = state + (dst,)
    elif kind == "other":
        state = state + (frozenset(),)
    if len(state) > CAP:
        state = (frozenset().union(*state[:len(state) - CAP + 1]),) + state[len(state) - CAP + 1:]
    return state


def check(path):
    lines = open(path).read().splitlines()
    bad = 0
    nfun = 0
    for name, body in functions(lines):
        nfun += 1
        bl = blocks(body)
        idx = {b[0]: i for i, b in enumerate(bl)}
        pred_state = {0: ()}
        work = [0]
        seen = {}
        issues = {}
        it = 0
        while work and it < 100000:
            it += 1
            k = work.pop()
            st = pred_state.get(k, ())
            if seen.get(k) == st:
                continue
            seen[k] = st
            for ln, s in bl[k][1]:
                st = step(st, s, lambda r, ln=ln, s=s: issues.setdefault(ln, (s, r)))
            for t in bl[k][2]:
                j = idx.get(t)
                if j is None:
                    continue
                m = merge(pred_state.get(j), st)
                if m != pred_state.get(j) or j not in seen:
                    pred_state[j] = m
                    work.append(j)
        for ln, (s, r) in sorted(issues.items()):
            print(f"{path}:{ln}: {name}: reads VGPR {r} of an LDS load still in flight: {s}")
            bad += 1
    print(f"{nfun} functions checked, {bad} reads of in-flight LDS destinations")
    return bad


if __name__ == "__main__":
    sys.exit(1 if sum(check(p) for p in sys.argv[1:]) else 0)
