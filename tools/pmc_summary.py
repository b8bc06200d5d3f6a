#!/usr/bin/env python3
"""Average each PMC counter per kernel over the dispatches in a tools/gpu_pmc.sh output dir."""
import collections
import csv
import glob
import os
import sys


def main(root, match=""):
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if match and match not in name:
                continue
            short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            agg[(short, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(agg.items()):
        print(f"{k[:60]:60s} {c:28s} n={len(v):3d} mean={sum(v) / len(v):.6g}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
