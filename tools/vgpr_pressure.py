#!/usr/bin/env python3
"""VGPR pressure map of one kernel from its gfx950 assembly (hipcc --save-temps .s file).

Backward liveness over the kernel's basic blocks (labels, s_branch / s_cbranch_* edges) on
physical VGPRs; a VALU / memory write counts as a killing definition (a write under a partial
EXEC mask is treated the same, so the count is a lower bound where lanes diverge).  Prints the
peak live-VGPR count, the instructions where it is reached, and for each source line (the .loc
directives) the largest live count seen -- where in the kernel's code the registers go.

usage: vgpr_pressure.py FILE.s KERNEL_SYMBOL [--top 20]"""
import argparse
import collections
import re

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
LABEL = re.compile(r"^(\.LBB\d+_\d+|\.Ltmp\d+):")


def regs(tok):
    out = set()
    for m in REG.finditer(tok):
        if m.group(1) is not None:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def parse(path, sym):
    lines, inside = [], False
    for ln in open(path):
        if ln.startswith(sym + ":"):
            inside = True
            continue
        if inside:
            if ln.strip().startswith(".Lfunc_end") or ln.startswith("\t.size\t" + sym):
                break
            lines.append(ln.rstrip("\n"))
    return lines


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("symbol")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    lines = parse(a.asm, a.symbol)
    files = {}
    for ln in open(a.asm):   # the .file table precedes the kernels
        p = ln.split()
        if len(p) >= 4 and p[0] == ".file" and p[1].isdigit():
            files[p[1]] = p[3].strip('"')
    # instructions with their block structure and source line
    insts, blocks, cur_loc = [], [], None
    labels = {}
    for ln in lines:
        s = ln.strip()
        m = LABEL.match(s)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        if s.startswith(".file"):
            p = s.split()
            if len(p) >= 3 and p[1].isdigit():
                files[p[1]] = p[3].strip('"') if len(p) >= 4 else p[-1].strip('"')
            continue
        if s.startswith(".loc"):
            p = s.split()
            cur_loc = (p[1], int(p[2]))
            continue
        if not s or s.startswith(".") or s.startswith(";"):
            continue
        s = s.split(";")[0].strip()
        mnem, _, ops = s.partition(" ")
        ops = [o.strip() for o in ops.split(",")] if ops else []
        defs, uses = set(), set()
        stores = mnem.startswith(("global_store", "buffer_store", "flat_store", "ds_write", "scratch_store",
                                  "global_atomic", "buffer_atomic", "ds_add", "ds_max", "ds_min"))
        no_vdst = mnem.startswith(("v_cmp", "v_readlane", "v_readfirstlane", "s_", "v_cmpx")) or stores
        for i, o in enumerate(ops):
            r = regs(o)
            if i == 0 and not no_vdst:
                if mnem.startswith("v_writelane"):
                    uses |= r
                defs |= r
            else:
                uses |= r
        if "_atomic" in mnem and ops and "glc" in s:   # returning atomics write their first operand
            defs |= regs(ops[0])
        insts.append((mnem, ops, defs, uses - defs if False else uses, cur_loc, s))
    n = len(insts)
    # basic block successors
    succ = collections.defaultdict(list)
    leaders = sorted(set([0] + list(labels.values())))
    for i, (mnem, ops, *_rest) in enumerate(insts):
        if mnem.startswith("s_branch") or mnem.startswith("s_cbranch"):
            tgt = ops[0] if ops else None
            if tgt in labels:
                succ[i].append(labels[tgt])
            if mnem.startswith("s_cbranch") and i + 1 < n:
                succ[i].append(i + 1)
        elif mnem in ("s_endpgm", "s_setpc_b64"):
            pass
        elif i + 1 < n:
            succ[i].append(i + 1)
    # iterative backward liveness per instruction (simple worklist)
    live_in = [set() for _ in range(n)]
    changed = True
    it = 0
    while changed and it < 200:
        changed = False
        it += 1
        for i in range(n - 1, -1, -1):
            out = set()
            for j in succ[i]:
                out |= live_in[j]
            _, _, d, u, _, _ = insts[i]
            new = (out - d) | u
            if new != live_in[i]:
                live_in[i] = new
                changed = True
    counts = [len(x) for x in live_in]
    peak = max(counts) if counts else 0
    print(f"{a.symbol}: {n} instructions, {it} liveness passes, peak live VGPRs {peak}")
    by_loc = collections.defaultdict(int)
    for i, c in enumerate(counts):
        loc = insts[i][4]
        if loc:
            by_loc[loc] = max(by_loc[loc], c)
    print("source lines by their largest live count:")
    for loc, c in sorted(by_loc.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"  {c:4d}  {files.get(loc[0], loc[0])}:{loc[1]}")
    def where(loc):
        return f"{files.get(loc[0], loc[0])}:{loc[1]}" if loc else "?"
    print("peak instructions:")
    shown = 0
    for i, c in enumerate(counts):
        if c >= peak - 1 and shown < a.top:
            shown += 1
            print(f"  {c:4d}  {insts[i][5][:90]}  ({where(insts[i][4])})")
    # the live set at the first peak: each register with the source lines of its reaching
    # definitions (backwards through the control flow graph)
    pred = collections.defaultdict(list)
    for i, js in succ.items():
        for j in js:
            pred[j].append(i)
    i0 = counts.index(peak)
    print(f"live at the first peak (instruction {i0}, {where(insts[i0][4])}):")
    groups = collections.defaultdict(list)
    for r in sorted(live_in[i0]):
        locs, seen, todo = set(), {i0}, list(pred[i0])
        while todo and len(locs) < 4:
            j = todo.pop()
            if j in seen:
                continue
            seen.add(j)
            if r in insts[j][2]:
                locs.add(where(insts[j][4]))
                continue
            todo.extend(pred[j])
        groups[" / ".join(sorted(locs)) or "?"].append(r)
    for w, rs in sorted(groups.items(), key=lambda kv: -len(kv[1])):
        print(f"  {len(rs):3d}  defined at {w}: v{rs}")


if __name__ == "__main__":
    main()
