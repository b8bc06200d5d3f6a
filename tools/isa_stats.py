"""Instruction mix of one kernel in a device .s file (hipcc --cuda-device-only -S).

usage: python tools/isa_stats.py file.s <mangled-name-substring> [--blocks]
Counts static instructions by class; with --blocks prints each basic block's size and
branch target so loops can be told apart from straight-line code."""
import re
import sys
from collections import Counter


def kernel_lines(path, key):
    out, on = [], False
    for ln in open(path):
        if not on and re.match(r"^_Z\S*%s\S*:" % re.escape(key), ln):
            on = True
            continue
        if on:
            if ln.startswith(".Lfunc_end"):
                break
            out.append(ln.rstrip())
    return out


def cls(op):
    for p in ("v_pk_", "v_mfma", "v_", "s_waitcnt", "s_", "global_load", "global_store", "global_atomic",
              "buffer_", "ds_", "flat_", "scratch_"):
        if op.startswith(p):
            return p
    return "other"


def main():
    path, key = sys.argv[1], sys.argv[2]
    lines = kernel_lines(path, key)
    c, blocks, cur, n = Counter(), [], None, 0
    for ln in lines:
        s = ln.strip()
        if not s or s.startswith(";") or s.startswith("."):
            if re.match(r"^\.LBB\S+:", s):
                if cur:
                    blocks.append((cur, n, last))
                cur, n, last = s[:-1], 0, ""
            continue
        op = s.split()[0]
        c[cls(op)] += 1
        c["total"] += 1
        n += 1
        last = s if op.startswith("s_cbranch") or op.startswith("s_branch") else ""
    if cur:
        blocks.append((cur, n, last))
    for k, v in c.most_common():
        print(f"{k:16s} {v}")
    if "--blocks" in sys.argv:
        for b, k, br in blocks:
            print(f"{b:12s} {k:5d} {br}")


if __name__ == "__main__":
    main()
