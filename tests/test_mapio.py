"""PIN map files: the reference's own ``pin_map.pth`` loads through the
safe loader (torch.load weights_only=True, nothing from the file executed), files written here
round-trip, the reference loads them back (when /root/reference is present, CPU), and a loaded
map answers SDF+gradient queries like the reference did on the saved map (GPU).

Fixture: tests/golden/pin_map_ref.pth, written by the reference's utils/tools.py:224-238
(save_implicit_map) in tests/golden/gen_golden.py, with the reference's outputs over that map in
pin_map_ref.npz.  SDF tolerance abs 1e-5 (north-star bar), gradients as test_gpu_parity.
"""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest
import torch

from pin_slam_amd import mapio

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF_FILE = os.path.join(GOLDEN, "pin_map_ref.pth")
REFERENCE = "/root/reference"


def _np(t):
    return t.detach().cpu().numpy()


def _check_map(nm, z):
    np.testing.assert_array_equal(_np(nm.neural_points), z["map_neural_points"])
    np.testing.assert_array_equal(_np(nm.point_orientations), z["map_point_orientations"])
    np.testing.assert_array_equal(_np(nm.geo_features), z["map_geo_features"])
    np.testing.assert_array_equal(_np(nm.point_ts_create), z["map_point_ts_create"])
    np.testing.assert_array_equal(_np(nm.point_ts_update), z["map_point_ts_update"])
    np.testing.assert_array_equal(_np(nm.point_certainties), z["map_point_certainties"])
    np.testing.assert_array_equal(_np(nm.travel_dist), z["map_travel_dist"])
    np.testing.assert_array_equal(_np(nm.local_mask), z["map_local_mask"])
    np.testing.assert_array_equal(_np(nm.global2local), z["map_global2local"])
    np.testing.assert_array_equal(_np(nm.local_geo_features), z["local_features"])
    np.testing.assert_array_equal(_np(nm.local_neural_points), z["local_neural_points"])
    table = _np(nm.buffer_pt_index)
    assert table.dtype == np.int32 and table.shape[0] == int(z["map_buffer_size"])
    slots = np.nonzero(table >= 0)[0]
    np.testing.assert_array_equal(slots, z["map_table_slots"])
    np.testing.assert_array_equal(table[slots], z["map_table_vals"])
    assert nm.cur_ts == int(z["map_cur_ts"])
    assert abs(nm.diff_travel_dist_local - float(z["map_diff_travel_dist_local"])) < 1e-6


def test_load_reference_map_file(golden):
    z = golden("pin_map_ref")
    d = mapio.load_pin_map(REF_FILE, device="cpu")
    _check_map(d["neural_points"], z)
    np.testing.assert_array_equal(_np(d["geo_decoder"]["layers.0.weight"]), z["dec_W1"])
    np.testing.assert_array_equal(_np(d["geo_decoder"]["lout.bias"]), z["dec_b2"])
    assert d["config"].query_nn_k == 8 and abs(d["config"].voxel_size_m - 0.3) < 1e-9


def test_loader_executes_nothing(tmp_path):
    """A map file naming any class outside the allow-list is refused, not imported."""
    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))
    p = tmp_path / "evil.pth"
    torch.save({"neural_points": Evil()}, p)
    with pytest.raises(Exception):
        mapio.load_pin_map(str(p), device="cpu")


def _roundtrip(tmp_path):
    from pin_slam_amd import Decoder
    d = mapio.load_pin_map(REF_FILE, device="cpu")
    dec = Decoder(d["config"], 64, 1, 1)
    dec.load_state_dict(d["geo_decoder"])
    path = mapio.save_implicit_map(str(tmp_path), d["neural_points"], dec, tensor_device="cpu")
    assert os.path.exists(os.path.join(str(tmp_path), "memory_footprint.npy"))
    return path


def test_save_roundtrip(golden, tmp_path):
    z = golden("pin_map_ref")
    path = _roundtrip(tmp_path)
    d2 = mapio.load_pin_map(path, device="cpu")
    _check_map(d2["neural_points"], z)
    np.testing.assert_array_equal(_np(d2["geo_decoder"]["layers.0.weight"]), z["dec_W1"])


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference tree not present")
def test_reference_loads_written_file(golden, tmp_path):
    """The reference's own torch.load + query path on a file written by save_implicit_map
    reproduces the reference's SDF on the original map (a file this package wrote, so a full
    unpickle is fine)."""
    path = _roundtrip(tmp_path)
    script = textwrap.dedent(f"""
        import sys, time, numpy as np, torch
        from unittest import mock
        sys.dont_write_bytecode = True
        for n in ["open3d", "roma", "wandb", "skimage", "skimage.measure", "natsort", "pyquaternion",
                  "pypose", "laspy", "gtsam", "evo"]:
            sys.modules[n] = mock.MagicMock(name=n)
        sys.path.insert(0, {REFERENCE!r})
        import utils.tools as T; T.get_time = time.time
        import model.neural_points as NP; NP.get_time = time.time
        from model.decoder import Decoder
        from model.neural_points import NeuralPoints
        m = torch.load({path!r}, weights_only=False)
        npm = m["neural_points"]
        assert type(npm) is NeuralPoints, type(npm)
        dec = Decoder(npm.config, npm.config.geo_mlp_hidden_dim, npm.config.geo_mlp_level, 1)
        dec.load_state_dict(m["geo_decoder"])
        z = np.load({os.path.join(GOLDEN, "pin_map_ref.npz")!r})
        for ql in (0, 1):
            feat, _, w, nnc, _ = npm.query_feature(torch.from_numpy(z["queries"]), training_mode=False,
                                                   query_locally=bool(ql))
            sdf = dec.sdf(feat).detach().numpy()
            assert np.array_equal(nnc.numpy(), z[f"q{{ql}}_nn_counts"])
            err = np.abs(sdf - z[f"q{{ql}}_sdf"]).max()
            assert err <= 1e-6, err
        print("ok")
    """)
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-3000:]


@pytest.mark.gpu
def test_loaded_map_queries_match_reference(golden):
    """Load the reference's file onto the GPU and run the fused SDF+grad query (both modes)."""
    from pin_slam_amd import Decoder, query_sdf
    from tests.test_gpu_parity import assert_grad_close
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    z = golden("pin_map_ref")
    d = mapio.load_pin_map(REF_FILE, device="cuda")
    nm = d["neural_points"]
    dec = Decoder(d["config"], 64, 1, 1)
    dec.load_state_dict(d["geo_decoder"])
    q = torch.as_tensor(z["queries"], device="cuda")
    for ql in (0, 1):
        sdf, grad, nn, _, _ = query_sdf(nm, dec, q, query_locally=bool(ql), want_grad=True)
        np.testing.assert_array_equal(_np(nn), z[f"q{ql}_nn_counts"])
        np.testing.assert_allclose(_np(sdf), z[f"q{ql}_sdf"], rtol=0, atol=1e-5)
        assert_grad_close(_np(grad), z[f"q{ql}_grad"])


@pytest.mark.gpu
def test_reference_save_path_pickles_the_live_object(tmp_path):
    """After install() the reference's own save_implicit_map (utils/tools.py:224-238) torch.saves
    the NeuralPoints object itself.  After map updates (capacity-buffer arrays, weak-reference
    caches) and a mapping() call, that pickle must work (NeuralPoints.__getstate__ drops the
    transient caches), store only each array's own rows, and load back to a map whose arrays and
    SDF queries equal the live map's."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import pin_slam_amd as P
    from pin_slam_amd.synthetic import surface_map, surface_pool, surface_scan
    nm, dec, pts = surface_map(200, device="cuda", buffer_size=1 << 22, query_backend="grid")
    nm.travel_dist = torch.arange(4, dtype=torch.float32, device="cuda")
    for k in range(3):
        nm.update(surface_scan(20.0 + k, 30.0, 8.0, 4096, seed=k, device="cuda"),
                  torch.tensor([20.0 + k, 30.0, 1.7], device="cuda"), None, k)
    coord, label, ts = surface_pool(pts, 20000, device="cuda")
    mapper = P.Mapper(nm.config, None, nm, dec)
    mapper.set_pool(coord, label, ts)
    mapper.mapping(2)
    assert nm.__dict__.get("_row_bufs"), "the map arrays should live in capacity buffers here"
    q = pts[::7].to("cuda").contiguous()
    want = P.query_sdf(nm, dec, q, query_locally=False, want_grad=True, want_certainty=False)
    os.makedirs(tmp_path / "model")
    path = str(tmp_path / "model" / "pin_map.pth")
    torch.save({"neural_points": nm, "geo_decoder": dec.state_dict()}, path)   # the reference's call
    assert os.path.getsize(path) < 2 * (nm.buffer_pt_index.numel() * 4 + 64 * nm.count() * 4 + (1 << 20))
    m = torch.load(path, weights_only=False)    # a file this test wrote
    back = m["neural_points"]
    for k in ("neural_points", "geo_features", "point_certainties", "point_ts_update", "local_neural_points",
              "local_geo_features", "global2local", "buffer_pt_index"):
        assert torch.equal(getattr(back, k), getattr(nm, k)), k
        t = getattr(back, k)
        assert t.untyped_storage().nbytes() == t.numel() * t.element_size(), k
    got = P.query_sdf(back, dec, q, query_locally=False, want_grad=True, want_certainty=False)
    assert torch.equal(got[0], want[0]) and torch.equal(got[1], want[1]) and torch.equal(got[2], want[2])
