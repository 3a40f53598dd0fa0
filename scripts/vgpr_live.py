#!/usr/bin/env python3
"""Approximate VGPR liveness of one kernel in a gfx950 .s file: where the
register pressure peaks (the allocation sets occupancy).

  hipcc --cuda-device-only -S ... -o k.s
  python3 scripts/vgpr_live.py k.s <mangled-kernel-name> [top]

Backward dataflow over the basic blocks of the listing; an instruction's first
VGPR operand is its def except for stores / no-return atomics / v_cmp /
v_readlane / s_* (uses only); v_writelane and 16-bit/SDWA partial writes keep
the old value live.  Prints the peak live count with the source lines around
it (the .s carries `; file:line` comments when built with -g0 -gline-tables-only).
"""
import re
import sys

VRE = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
NO_DEF = ("global_store", "buffer_store", "ds_write", "ds_add_u32", "ds_sub_u32", "ds_or_b32", "ds_max",
          "ds_min", "ds_and", "ds_xor", "flat_store", "scratch_store", "v_cmp", "v_cmpx", "v_readlane",
          "v_readfirstlane", "s_")


def regs(tok):
    out = []
    for m in VRE.finditer(tok):
        if m.group(3) is not None:
            out.append(int(m.group(3)))
        else:
            out.extend(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def parse(lines):
    blocks, cur, label = [], [], None
    for ln in lines:
        t = ln.split(";")[0].strip()
        if not t:
            continue
        if t.endswith(":") and not t.startswith("."):
            continue
        if re.match(r"^\.LBB\d+_\d+:", t):
            if cur or label is not None:
                blocks.append((label, cur))
            label, cur = t[:-1], []
            continue
        if t.startswith("."):
            continue
        cur.append(t)
        if t.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc")):
            blocks.append((label, cur))
            label, cur = None, []
    if cur:
        blocks.append((label, cur))
    return blocks


def defs_uses(ins):
    op = ins.split()[0]
    rest = ins[len(op):]
    parts = [p.strip() for p in rest.split(",")]
    if not parts or not parts[0]:
        return [], []
    if op.startswith(NO_DEF) or ("atomic" in op and " sc0" not in ins and "glc" not in ins):
        return [], regs(rest)
    d = regs(parts[0])
    u = regs(",".join(parts[1:]))
    if op.startswith("v_writelane") or "sdwa" in op or "_d16" in op or op.startswith("v_mov_b32_dpp"):
        u += d
    return d, u


def main():
    path, name = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    s = open(path).read()
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    lines = s[i:j].splitlines()[1:]
    blocks = parse(lines)
    idx = {lab: k for k, (lab, _) in enumerate(blocks) if lab}
    succ = []
    for k, (lab, ins) in enumerate(blocks):
        sc = []
        last = ins[-1] if ins else ""
        m = re.search(r"(\.LBB\d+_\d+)", last)
        if last.startswith(("s_branch", "s_cbranch")) and m:
            sc.append(idx[m.group(1)])
        if not last.startswith(("s_branch", "s_endpgm", "s_setpc")) and k + 1 < len(blocks):
            sc.append(k + 1)
        succ.append(sc)
    live_in = [set() for _ in blocks]
    changed = True
    while changed:
        changed = False
        for k in range(len(blocks) - 1, -1, -1):
            out = set()
            for t in succ[k]:
                out |= live_in[t]
            for ins in reversed(blocks[k][1]):
                d, u = defs_uses(ins)
                out -= set(d)
                out |= set(u)
            if out != live_in[k]:
                live_in[k] = out
                changed = True
    peaks = []
    for k, (lab, ins) in enumerate(blocks):
        out = set()
        for t in succ[k]:
            out |= live_in[t]
        per = []
        for ins_ in reversed(ins):
            d, u = defs_uses(ins_)
            per.append((len(out | set(d)), ins_))
            out -= set(d)
            out |= set(u)
        for n, ins_ in reversed(per):
            peaks.append((n, k, lab, ins_))
    peaks.sort(key=lambda x: -x[0])
    print("blocks", len(blocks), "peak live VGPRs", peaks[0][0])
    seen = set()
    for n, k, lab, ins_ in peaks:
        if k in seen:
            continue
        seen.add(k)
        print("%4d  block %-12s %s" % (n, lab, ins_[:90]))
        if len(seen) >= top:
            break


if __name__ == "__main__":
    main()
