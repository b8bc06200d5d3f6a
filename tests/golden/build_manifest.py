#!/usr/bin/env python3
"""(Re)build GENERATED_WITH.json for fixtures that predate the per-fixture record (gen_golden.py's
record_fixture writes an entry whenever it generates a fixture): per .npz file the generating call,
the date of the commit that last changed it, the library versions of the image it was made in
(torch 2.10.0+rocm7.0, numpy 2.2.6 -- the only image this repository has used), the torch thread
count where the fixture stores it, its SHA-256, and for the SLAM replays the envelope runs.
Existing entries are kept unless --force.  Needs no reference import.

Usage: python tests/golden/build_manifest.py [--force]
"""
import glob
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
MANIFEST = os.path.join(HERE, "GENERATED_WITH.json")
GENERATORS = {
    "neighborhoods": "gen_golden.py gen_neighborhoods",
    "query_wf": "gen_golden.py gen_query_case('query_wf', weighted_first=True, seed=1)",
    "query_nwf": "gen_golden.py gen_query_case('query_nwf', weighted_first=False, seed=2)",
    "query_kitti": "gen_golden.py gen_query_case('query_kitti', voxel 0.4, alpha 0.5, k 6, seed=3)",
    "query_ties": "gen_golden.py query_ties (lattice map and queries, voxel 0.25, alpha 0.5, seed=16)",
    "mapper_wf": "gen_golden.py gen_mapper_case('mapper_wf', seed=4)",
    "mapper_nwf": "gen_golden.py gen_mapper_case('mapper_nwf', seed=5)",
    "tracker_wf": "gen_golden.py tracker_wf",
    "tracker_nwf": "gen_golden.py tracker_nwf",
    "mesher_wf": "gen_golden.py gen_mesher_case('mesher_wf', seed=8)",
    "map_seq": "gen_golden.py map_seq",
    "map_seq_mid": "gen_golden.py map_seq_mid",
    "pin_map_ref": "gen_golden.py pin_map_ref",
    "sampler_default": "gen_golden.py sampler",
    "sampler_dropoff": "gen_golden.py sampler",
    "process_frame": "gen_golden.py process_frame",
    "slam_seq": "gen_golden.py slam_seq + gen_slam_envelope.py run/combine slam_seq",
    "slam_seq100": "gen_golden.py slam_seq100 + gen_slam_envelope.py run/combine slam_seq100",
}


def _commit_date(path):
    out = subprocess.run(["git", "log", "-1", "--format=%cs", "--", path], capture_output=True, text=True,
                         cwd=HERE).stdout.strip()
    return out or "uncommitted"


def main(force=False):
    m = json.load(open(MANIFEST)) if os.path.exists(MANIFEST) else {}
    for path in sorted(glob.glob(os.path.join(HERE, "*.npz"))):
        name = os.path.basename(path)
        stem = name[:-4]
        if name in m and not force:
            continue
        z = np.load(path, allow_pickle=False)
        e = dict(generator=GENERATORS.get(stem, "gen_golden.py mapping_calls" if stem.startswith("mapping_") else "?"),
                 generated=_commit_date(path), torch="2.10.0+rocm7.0", numpy="2.2.6",
                 sha256=hashlib.sha256(open(path, "rb").read()).hexdigest())
        if "torch_threads" in z.files:
            e["torch_threads"] = int(z["torch_threads"])
        if "env_threads" in z.files:
            e["envelope_runs"] = [str(v) for v in z["env_labels"]]
            e["envelope_generated"] = str(z["env_generated"])
        m[name] = e
    with open(MANIFEST, "w") as f:
        json.dump(dict(sorted(m.items())), f, indent=1)
        f.write("\n")
    print(len(m), "fixtures in", MANIFEST)


def update(stem, **fields):
    """Set fields of one fixture's entry (gen_slam_envelope.py combine), the SHA-256 refreshed."""
    m = json.load(open(MANIFEST)) if os.path.exists(MANIFEST) else {}
    path = os.path.join(HERE, f"{stem}.npz")
    e = m.get(f"{stem}.npz", {})
    e.update(fields, sha256=hashlib.sha256(open(path, "rb").read()).hexdigest())
    m[f"{stem}.npz"] = e
    with open(MANIFEST, "w") as f:
        json.dump(dict(sorted(m.items())), f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main("--force" in sys.argv)
