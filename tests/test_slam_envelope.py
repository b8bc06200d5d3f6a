"""The SLAM replay's bounds (tests/test_gpu_slam.py) against the reference alone, on the CPU:
every reference run stored in a fixture's envelope (env_*, tests/golden/gen_slam_envelope.py) must
pass the same pose, count and surface checks when judged against the OTHER runs of that fixture
(leave-one-out).  This is how the widening factors were calibrated; it also shows they are not
slack: at factor 1 some reference runs fail."""
import numpy as np
import pytest

from tests import test_gpu_slam as S

FIXTURES = ["slam_seq", "slam_seq100"]


def _without(z, r):
    R = np.asarray(z["env_hist_pose"]).shape[0]
    return {k: (np.delete(v, r, 0) if k.startswith("env_") and np.ndim(v) > 0 and np.shape(v)[0] == R else v)
            for k, v in z.items()}


def _failures(z, r):
    zz = _without(z, r)
    penv = S.pose_envelope(zz)
    out = []
    for k in range(int(z["frames"])):
        if not S.pose_check(np.asarray(z["env_hist_pose"][r, k], np.float64), k, penv)[0]:
            out.append(f"pose {k}")
        for name, floor in S.COUNT_FLOORS.items():
            if not S.count_check(z[f"env_hist_{name}"][r, k], zz[f"env_hist_{name}"][:, :k + 1], floor)[0]:
                out.append(f"{name} {k}")
    for key in ("f0_surface_sdf", "end_surface_sdf"):
        if not S.surface_bounds(z["env_" + key][r], zz["env_" + key])[0]:
            out.append(key)
    return out


@pytest.mark.parametrize("fixture", FIXTURES)
def test_every_reference_run_passes_against_the_others(golden, fixture):
    z = dict(golden(fixture))
    R = np.asarray(z["env_hist_pose"]).shape[0]
    assert R >= 7, "the envelope holds at least 7 reference runs"
    bad = {str(z["env_labels"][r]): f for r in range(R) if (f := _failures(z, r))}
    assert not bad, bad


def test_factors_are_not_slack(golden, monkeypatch):
    """With every factor at 1 (the envelope of the other runs, unwidened) some reference run fails:
    the calibrated factors are what the reference's own run-to-run scatter needs."""
    monkeypatch.setattr(S, "W_POSE", 1.0)
    monkeypatch.setattr(S, "W_COUNT", 1.0)
    monkeypatch.setattr(S, "W_SURFACE", 1.0)
    fails = 0
    for fixture in FIXTURES:
        z = dict(golden(fixture))
        fails += sum(bool(_failures(z, r)) for r in range(np.asarray(z["env_hist_pose"]).shape[0]))
    assert fails > 0
