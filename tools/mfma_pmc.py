#!/usr/bin/env python3
"""Per-kernel means of the tools/mfma_pmc.sh counters for the SDF kernels -> JSON: MFMA
instructions and F16 FLOPs per launch, matrix-core busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over
GRBM_GUI_ACTIVE x 1024 SIMDs, the MfmaUtil derived metric of rocprofv3 -L)."""
import collections
import csv
import glob
import json
import os
import subprocess
import sys

SIMDS = 1024   # 256 CUs x 4 SIMDs


def main(root):
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            if "k_query_sdf" not in name:
                continue
            agg[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
    kernels = {}
    for (name, c), v in agg.items():
        kernels.setdefault(name, {})[c] = sum(v) / len(v)
    out = []
    for name, c in sorted(kernels.items()):
        busy, act = c.get("SQ_VALU_MFMA_BUSY_CYCLES"), c.get("GRBM_GUI_ACTIVE")
        out.append({"name": name, "mfma_insts": c.get("SQ_INSTS_MFMA"),
                    "f16_flop": c["SQ_INSTS_VALU_MFMA_MOPS_F16"] * 512 if "SQ_INSTS_VALU_MFMA_MOPS_F16" in c else None,
                    "mfma_busy_cycles": busy, "gui_active_cycles": act,
                    "mfma_util": busy / (act * SIMDS) if busy is not None and act else None})
    rev = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
    json.dump({"commit": rev or None, "kernels": out}, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
