#!/usr/bin/env python3
"""Time the mapper leg of bench.py for each library in tools/exp_libs (GPU box)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "exp_libs")
for rep in range(2):
    for lib in sorted(f for f in os.listdir(OUT) if f.endswith(".so")):
        env = dict(os.environ, PIN_LIB=os.path.join(OUT, lib))
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--steps", "5",
                            "--no-tracker", "--no-mesher", "--no-map-update", "--no-process-frame"],
                           env=env, capture_output=True, text=True, timeout=400)
        if r.returncode:
            print(lib, "FAILED", r.stderr[-1500:])
            sys.exit(1)
        d = json.loads(r.stdout.strip().splitlines()[-1])["mapper"]
        print(f"rep{rep} {lib:20s} {d['value']:.1f} it/s  {d['ms_per_iter']:.3f} ms/iter", flush=True)
