"""isa_mix.py -- VALU issue-class count of a kernel's hot loops.

Reads the device assembly that `make -C volsync_amd/csrc asm` leaves in
volsync_amd/lib/obj (--save-temps), splits it into kernels, finds every loop
(the compiler marks each header "Loop Header: Depth=N"; the body runs from the
header to the last branch back to it) and counts the instructions of a loop's
body by mnemonic, pricing each VALU instruction with the issue cost measured on
MI355X (tools/valu/valu_ops*.hip -> profiles/r03_start/valu_ops*.json,
profiles/r02_valu_peak): shader cycles per wave-instruction per SIMD at 8 waves
per SIMD.  Two classes dominate:
  ~2.3 cycles: v_xor/v_and/v_or/v_add_u32/v_sub_u32/v_mov_b32/v_lshrrev_b32,
               v_bitop3_b32 whose sources are VGPRs or inline constants;
  ~4.2 cycles: v_alignbit/v_alignbyte/v_perm/v_add3/v_and_or/v_lshl_or/
               v_lshlrev_b32/v_bfe/v_min_u32, DPP/SDWA forms, v_bitop3_b32
               reading an SGPR, 64-bit shifts/adds;
  v_cndmask_b32: 4.25 as _e64 with an SGPR-pair mask, ~2.3 as _e32 reading the
  VCC a v_cmp just wrote (the pair averages 3.3; profiles/r05_start/valu_ops3.json).
The output is the issue-cycle floor of one trip of the loop, per wave:
python tools/isa_mix.py volsync_amd/lib/obj/sha256-hip-amdgcn-amd-amdhsa-gfx950.s sha_slice_kernel
"""
from __future__ import annotations

import argparse
import json
import re
import sys
from collections import Counter

# measured (8 waves per SIMD) -- see the docstring for the sources
FAST = 2.3
SLOW = 4.2
COST = {
    "v_xor_b32": FAST, "v_and_b32": FAST, "v_or_b32": FAST, "v_add_u32": FAST,
    "v_sub_u32": FAST, "v_subrev_u32": FAST, "v_mov_b32": FAST, "v_lshrrev_b32": FAST,
    "v_lshlrev_b16": FAST, "v_fma_f32": FAST, "v_not_b32": FAST,
    "v_alignbit_b32": SLOW, "v_alignbyte_b32": SLOW, "v_perm_b32": SLOW, "v_add3_u32": SLOW,
    "v_and_or_b32": SLOW, "v_lshl_or_b32": SLOW, "v_lshlrev_b32": SLOW, "v_bfe_u32": SLOW,
    "v_min_u32": SLOW, "v_min3_u32": SLOW, "v_max_u32": SLOW, "v_or3_b32": SLOW,
    "v_xad_u32": SLOW, "v_bfi_b32": SLOW, "v_lshl_add_u32": SLOW, "v_add_lshl_u32": SLOW,
    "v_mul_lo_u32": SLOW, "v_mul_hi_u32": SLOW, "v_dot4_u32_u8": SLOW, "v_bfrev_b32": SLOW,
    "v_lshrrev_b64": SLOW, "v_lshlrev_b64": SLOW, "v_lshl_add_u64": SLOW,
    "v_add_co_u32": SLOW, "v_addc_co_u32": SLOW, "v_pk_mov_b32": SLOW, "v_pk_add_u16": SLOW,
    "v_min3_u16": 8.2, "v_cndmask_b32": FAST,
}

LABEL_RE = re.compile(r"^(\.LBB\d+_\d+):")
INSN_RE = re.compile(r"^\s+([sv]_\w+|ds_\w+|global_\w+|buffer_\w+|flat_\w+|scratch_\w+)\b(.*)$")


def kernels(lines):
    """{kernel symbol: (first line, last line)} from the .s text."""
    out = {}
    cur = None
    for i, ln in enumerate(lines):
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            cur = m.group(1)
            out[cur] = [i, i]
        elif cur and re.match(r"^\s*\.Lfunc_end", ln):
            out[cur][1] = i
            cur = None
    return out


def classify(mn: str, ops: str):
    base = mn.split("_e32")[0].split("_e64")[0]
    if mn.startswith("v_"):
        if "_dpp" in mn or "_sdwa" in mn or "row_" in ops or "quad_perm" in ops:
            return "valu", SLOW
        if base == "v_bitop3_b32":
            srcs = [s.strip() for s in ops.split(",")[1:4]]
            return "valu", SLOW if any(re.match(r"^(s\d|s\[|vcc|exec)", s) for s in srcs) else FAST
        if base in ("v_readfirstlane_b32", "v_readlane_b32", "v_writelane_b32"):
            return "valu", SLOW
        if base == "v_cndmask_b32":
            return "valu", SLOW if mn.endswith("_e64") else FAST
        if base.startswith("v_cmp") or base.startswith("v_cmpx"):
            return "valu", SLOW
        return "valu", COST.get(base, SLOW)
    if mn.startswith("ds_"):
        return "lds", 0.0
    if mn.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem", 0.0
    if mn.startswith("s_"):
        return "salu", 0.0
    return "other", 0.0


def loops(lines, lo, hi):
    """{header label: {"depth", "parent", "blocks": [(first, last)]}} for the loops of
    lines[lo:hi]: every basic block carries the compiler's note of its innermost
    loop ("in Loop: Header=BBx_y", or "Loop Header" on the header itself)."""
    blocks = []  # (label, first, last, innermost header, depth, parent)
    cur = None
    for i in range(lo, hi):
        ln = lines[i]
        m = LABEL_RE.match(ln) or re.match(r"^; %bb\.(\d+):", ln)
        if m:
            if cur:
                cur[2] = i - 1
                blocks.append(cur)
            lab = m.group(1) if ln.startswith(".LBB") else None
            cur = [lab, i, i, None, 0, None]
        if cur is None:
            continue
        h = re.search(r"Loop Header: Depth=(\d+)", ln)
        if h and cur[0]:
            cur[3], cur[4] = cur[0], int(h.group(1))
        p = re.search(r"Parent Loop BB(\d+_\d+) Depth=(\d+)", ln)
        if p and cur[3] == cur[0] and cur[5] is None:
            cur[5] = ".LBB" + p.group(1)
        n = re.search(r"in Loop: Header=BB(\d+_\d+) Depth=(\d+)", ln)
        if n and cur[3] is None:
            cur[3], cur[4] = ".LBB" + n.group(1), int(n.group(2))
    if cur:
        cur[2] = hi - 1
        blocks.append(cur)
    out = {}
    for lab, first, last, head, depth, parent in blocks:
        if head is None:
            continue
        e = out.setdefault(head, {"depth": depth, "parent": None, "blocks": []})
        if lab == head:
            e["depth"], e["parent"] = depth, parent
        e["blocks"].append((first, last))
    return out


def count(lines, ranges):
    mn = Counter()
    cyc = 0.0
    cls = Counter()
    for i in (i for first, last in ranges for i in range(first, last + 1)):
        m = INSN_RE.match(lines[i])
        if not m:
            continue
        name, ops = m.group(1), m.group(2)
        c, w = classify(name, ops)
        mn[name] += 1
        cls[c] += 1
        if c == "valu":
            cyc += w
            cls["valu_fast" if w <= FAST else "valu_slow"] += 1
    return mn, cls, cyc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel", help="substring of the kernel's symbol")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    lines = open(a.asm).read().splitlines()
    ks = {k: v for k, v in kernels(lines).items() if a.kernel in k}
    res = {}
    for k, (lo, hi) in ks.items():
        res[k] = []
        ls = loops(lines, lo, hi)
        for lab, e in sorted(ls.items(), key=lambda x: x[1]["blocks"][0][0]):
            # own blocks only: a child loop's blocks are reported under the child
            mn, cls, cyc = count(lines, e["blocks"])
            kids = [c for c, ce in ls.items() if ce["parent"] == lab]
            res[k].append({"loop": lab, "depth": e["depth"], "parent": e["parent"],
                           "children": kids, "lines": e["blocks"][0][0] + 1,
                           "classes": dict(cls), "valu_issue_cycles": round(cyc, 1),
                           "top": mn.most_common(a.top)})
    if a.json:
        json.dump(res, sys.stdout, indent=1)
        print()
        return
    for k, ls in res.items():
        print(k)
        for r in ls:
            print(f"  loop {r['loop']} depth {r['depth']} at line {r['lines']} children "
                  f"{r['children']}: {r['classes']} "
                  f"valu issue {r['valu_issue_cycles']} cycles")
            for name, n in r["top"]:
                print(f"      {n:6d} {name}")


if __name__ == "__main__":
    main()
