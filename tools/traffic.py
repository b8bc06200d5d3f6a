#!/usr/bin/env python3
"""Per-kernel mean FETCH_SIZE / WRITE_SIZE (KB per dispatch) from tools/traffic.sh output ->
bytes per launch.  gfx950: FETCH_SIZE tallies 128-B requests at 64 B (MI355X_MICROARCH.md,
HBM section), so it is doubled; WRITE_SIZE is taken as reported."""
import collections
import csv
import glob
import json
import os
import subprocess
import sys


def main(root):
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
            agg[(name.split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    kernels = {}
    for (name, c), v in agg.items():
        kernels.setdefault(name, {})[c] = sum(v) / len(v)
    out = []
    for name, c in sorted(kernels.items()):
        if "FETCH_SIZE" not in c:
            continue
        fetch = 2 * c["FETCH_SIZE"] * 1024
        write = c.get("WRITE_SIZE", 0.0) * 1024
        out.append({"name": name, "fetch_kb_raw": c["FETCH_SIZE"], "write_kb": c.get("WRITE_SIZE"),
                    "bytes_per_launch": fetch + write})
    rev = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
    json.dump({"commit": rev or None, "kernels": out}, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
