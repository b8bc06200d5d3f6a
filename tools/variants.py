#!/usr/bin/env python3
"""Build compile-time variants of the library (here) and time them (on the GPU box).

    python tools/variants.py build NAME=-DFLAG=1,-DOTHER=0 NAME2=...   # writes tools/exp_libs/NAME.so
    python tools/variants.py run [bench args]                          # one bench per variant, same box
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "exp_libs")


def build(specs):
    sys.path.insert(0, ROOT)
    from pin_slam_amd import build as B
    os.makedirs(OUT, exist_ok=True)
    for spec in specs:
        name, _, flags = spec.partition("=")
        extra = [f for f in flags.split(",") if f]
        B.build(force=True, extra=extra, out=os.path.join(OUT, name + ".so"))
        print("built", name, extra)


def run(args):
    libs = sorted(f for f in os.listdir(OUT) if f.endswith(".so"))
    for rep in range(2):
        for lib in libs:
            env = dict(os.environ, PIN_LIB=os.path.join(OUT, lib))
            legs = [] if os.environ.get("VAR_MAPPER") else ["--no-mapper"]
            legs += [] if os.environ.get("VAR_NWF") else ["--no-nwf-leg"]
            r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *legs, "--no-cpu-baseline",
                                "--no-tracker", "--no-mesher", "--no-map-update", "--no-process-frame", "--no-slam", "--no-mapper-nwf", *args],
                               env=env, capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(lib, "FAILED", r.stderr[-2000:])
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            print(f"rep{rep} {lib:24s} {d['value'] / 1e9:.3f} Gq/s  kernel {d['roofline']['kernel_ms'] * 1e3:.1f} us  order {d['roofline'].get('order_pass_ms', 0) * 1e3:.1f} us"
                  + (f"  mapper {d['mapper']['value']:.1f} it/s" if "mapper" in d else "")
                  + (f"  per-neighbour {d['per_neighbour']['value'] / 1e9:.3f} Gq/s" if "per_neighbour" in d else ""),
                  flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        run(sys.argv[2:])
