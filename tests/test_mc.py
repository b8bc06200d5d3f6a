"""Marching cubes for Mesher.mc_mesh.

PARITY UNPINNED against the reference: utils/mesher.py:327 calls skimage.measure.marching_cubes
(Lewiner), and skimage is not installed here, so neither its tables nor its outputs are
available.  What is checked: the generated kernel table equals the oracle's independent
construction; the kernel equals the oracle exactly (vertex positions, face lists, masks) on
small grids; on sphere SDFs the surface is closed (every edge in exactly two faces, Euler
characteristic 2), vertices lie on the sphere to the linear-interpolation error, and normals
point outward.
"""
import os
import re

import numpy as np
import pytest
import torch

from oracle import pin_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_table():
    txt = open(os.path.join(ROOT, "pin_slam_amd", "csrc", "pin_mc_table.h")).read()
    rows = re.findall(r"\{([-0-9, ]+)\}", txt)
    assert len(rows) == 256
    out = []
    for r in rows:
        vals = [int(v) for v in r.split(",")]
        tri = []
        for i in range(0, len(vals) - 1, 3):
            if vals[i] < 0:
                break
            tri.append(tuple(vals[i:i + 3]))
        out.append(tri)
    return out


def test_kernel_table_matches_oracle_construction():
    hdr = _header_table()
    for c in range(256):
        assert hdr[c] == O.mc_case_triangles(c), c
    # complementary patterns give the same triangles reversed, except on ambiguous faces
    assert O.mc_case_triangles(0) == [] and O.mc_case_triangles(255) == []


def _sphere(n, r, c=None):
    c = np.full(3, (n - 1) / 2.0) if c is None else np.asarray(c)
    g = np.stack(np.meshgrid(*[np.arange(n)] * 3, indexing="ij"), -1).astype(np.float64)
    return (np.linalg.norm(g - c, axis=-1) - r).astype(np.float32)


def _closed_mesh_checks(verts, faces, centre):
    e = np.sort(np.concatenate([faces[:, [0, 1]], faces[:, [1, 2]], faces[:, [2, 0]]]), 1)
    _, cnt = np.unique(e, axis=0, return_counts=True)
    assert (cnt == 2).all(), "open or non-manifold edges"
    V, E, F = len(np.unique(faces)), len(cnt), len(faces)
    assert V - E + F == 2
    p = verts[faces]
    n = np.cross(p[:, 1] - p[:, 0], p[:, 2] - p[:, 0])
    out = ((p.mean(1) - centre) * n).sum(1)
    assert (out > 0).mean() > 0.99, "normals should point from inside (< level) to outside"


def test_oracle_sphere_closed():
    v = _sphere(14, 4.3)
    verts, faces = O.marching_cubes(v)
    _closed_mesh_checks(verts, faces, np.full(3, 6.5))
    r = np.linalg.norm(verts - 6.5, axis=1)
    assert np.abs(r - 4.3).max() < 0.1


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return "cuda"


@pytest.mark.gpu
@pytest.mark.parametrize("with_mask", [False, True])
def test_kernel_matches_oracle(dev, with_mask):
    from pin_slam_amd.mesher import marching_cubes
    rng = np.random.default_rng(3)
    v = _sphere(16, 5.1, c=(7.3, 7.9, 6.6)) + rng.normal(0, 0.3, (16, 16, 16)).astype(np.float32)
    v[3, 4, 5] = 0.0                      # exactly on the level: degenerate triangles appear
    mask = rng.random((16, 16, 16)) > 0.3 if with_mask else None
    want_v, want_f = O.marching_cubes(v, mask)
    got_v, got_f = marching_cubes(torch.as_tensor(v, device=dev), None if mask is None else torch.as_tensor(mask,
                                  device=dev), allow_degenerate=True)
    np.testing.assert_array_equal(got_v.cpu().numpy(), want_v)
    np.testing.assert_array_equal(got_f.cpu().numpy(), want_f)


@pytest.mark.gpu
def test_kernel_sphere_closed_and_mc_mesh(dev):
    import pin_slam_amd as P
    from pin_slam_amd.mesher import marching_cubes
    v = _sphere(96, 30.2, c=(47.1, 46.7, 47.9))
    verts, faces = marching_cubes(torch.as_tensor(v, device=dev))
    verts, faces = verts.cpu().numpy(), faces.cpu().numpy()
    _closed_mesh_checks(verts, faces, np.array([47.1, 46.7, 47.9]))
    assert np.abs(np.linalg.norm(verts - [47.1, 46.7, 47.9], axis=1) - 30.2).max() < 0.05
    # the drop-in mc_mesh: world coordinates like utils/mesher.py:335
    m = P.Mesher(P.Config(device=dev), None, None)
    wv, wf = m.mc_mesh(v, None, 0.1, np.array([1.0, 2.0, 3.0]))
    np.testing.assert_allclose(wv, np.array([1.0, 2.0, 3.0]) + verts.astype(np.float64) * 0.1)
    np.testing.assert_array_equal(wf, faces)


@pytest.mark.gpu
def test_kernel_edge_cases(dev):
    from pin_slam_amd.mesher import marching_cubes
    v = torch.ones((5, 6, 7), device=dev)
    verts, faces = marching_cubes(v)                     # no crossing
    assert verts.shape == (0, 3) and faces.shape == (0, 3)
    v[2, 3, 3] = -1.0
    verts, faces = marching_cubes(v, torch.zeros((5, 6, 7), dtype=torch.bool, device=dev))   # all masked
    assert faces.shape[0] == 0
    verts, faces = marching_cubes(v)                     # one inside point: a closed octahedron-like cell
    assert faces.shape[0] == 8 and verts.shape[0] == 6
    with pytest.raises(ValueError):
        marching_cubes(torch.ones((1, 4, 4), device=dev))
    # the drop-in mc_mesh returns an empty mesh instead (the reference's try/except,
    # utils/mesher.py:324-333)
    import pin_slam_amd as P
    m = P.Mesher(P.Config(device=dev), None, None)
    wv, wf = m.mc_mesh(np.ones((1, 4, 4), np.float32), None, 0.1, np.array([1.0, 2.0, 3.0]))
    assert wv.shape == (0, 3) and wf.shape == (0, 3)
