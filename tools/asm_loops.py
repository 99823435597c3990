#!/usr/bin/env python3
"""Static loop census of one kernel in the gfx950 assembly (make -C rvgrt_amd/csrc asm).

    python tools/asm_loops.py <mangled-name-substring> [rv_kernels.s]

Finds the kernel's body, every backward branch (a loop: target label at or
before the branch) and prints, per loop, its line range and the VALU / SALU /
vector-memory / LDS / branch instruction counts of the instructions between
the target label and the branch (the loop body as laid out, inner loops
included).  Used to price a traversal step in instructions before measuring.
"""
import re
import sys


def classify(op):
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_rd"
    if op.startswith(("global_store", "buffer_store", "flat_store", "global_atomic")):
        return "vmem_wr"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    return None


def main():
    key = sys.argv[1]
    path = sys.argv[2] if len(sys.argv) > 2 else "rvgrt_amd/csrc/build/rv_kernels.s"
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^[A-Za-z_][\w.]*:", l) and key in l.split(":")[0]:
            start = i
            break
    if start is None:
        sys.exit(f"no kernel matching {key}")
    end = start + 1
    while end < len(lines) and not lines[end].startswith("\t.section") and ".Lfunc_end" not in lines[end]:
        end += 1
    body = lines[start:end]
    labels = {}
    insts = []   # (line index in body, op, label-target or None)
    for i, l in enumerate(body):
        s = l.strip()
        if re.match(r"^\.LBB\d+_\d+:", s):
            labels[s[:-1].split(":")[0]] = i
            continue
        if not s or s.startswith((";", ".", "//")):
            continue
        op = s.split()[0]
        tgt = None
        if op.startswith(("s_cbranch", "s_branch")):
            m = re.search(r"(\.LBB\d+_\d+)", s)
            tgt = m.group(1) if m else None
        insts.append((i, op, tgt))
    tot = {}
    for _, op, _ in insts:
        c = classify(op)
        if c:
            tot[c] = tot.get(c, 0) + 1
    print(f"{body[0]} lines {start + 1}-{end}: {tot}")
    for i, op, tgt in insts:
        if tgt and tgt in labels and labels[tgt] <= i:
            lo = labels[tgt]
            cnt = {}
            for j, op2, _ in insts:
                if lo <= j <= i:
                    c = classify(op2)
                    if c:
                        cnt[c] = cnt.get(c, 0) + 1
            print(f"  loop {tgt} body lines {start + lo + 1}-{start + i + 1} ({op}): {cnt}")


if __name__ == "__main__":
    main()
