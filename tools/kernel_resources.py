#!/usr/bin/env python3
"""Print per-kernel VGPR/SGPR/spill/occupancy from hipcc's resource-usage remarks."""
import re
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(src):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "pin_slam_amd", "csrc"), "-c", src,
           "-o", "/tmp/_kr.o", "--offload-device-only", "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
        if not m:
            continue
        key, val = m.group(1).strip(), m.group(2).strip()
        if key == "Function Name":
            cur = {"name": val}
            rows.append(cur)
        elif cur is not None:
            cur[key] = val
    for r in rows:
        name = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
        name = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
        print(f"{name:50s} VGPR {r.get('VGPRs','?'):>4s} AGPR {r.get('AGPRs','?'):>3s} SGPR {r.get('SGPRs','?'):>3s} "
              f"spillV {r.get('VGPRs Spill','?'):>3s} occ {r.get('Occupancy [waves/SIMD]','?'):>2s} "
              f"LDS {r.get('LDS Size [bytes/block]','?')}")


if __name__ == "__main__":
    main(sys.argv[1])
