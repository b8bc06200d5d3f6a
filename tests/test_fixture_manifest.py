"""Fixture provenance (tests/golden/GENERATED_WITH.json): every golden .npz has an entry naming
its generating call, date, torch / numpy versions, and the SHA-256 of the file as committed -- a
regenerated fixture without a refreshed entry fails here."""
import glob
import hashlib
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_every_fixture_has_a_current_entry():
    m = json.load(open(os.path.join(GOLDEN, "GENERATED_WITH.json")))
    files = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "*.npz")))
    assert sorted(m) == files
    for name in files:
        e = m[name]
        for k in ("generator", "generated", "torch", "numpy", "sha256"):
            assert e.get(k), (name, k)
        assert hashlib.sha256(open(os.path.join(GOLDEN, name), "rb").read()).hexdigest() == e["sha256"], name
    for name in ("slam_seq.npz", "slam_seq100.npz"):
        assert len(m[name]["envelope_runs"]) >= 7, name
