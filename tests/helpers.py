"""Shared test helpers: build the drop-in classes from golden fixtures / synthetic maps."""
import numpy as np
import torch

import pin_slam_amd as P
from oracle import pin_oracle as O


def config_from_fixture(z, device="cuda", backend="auto"):
    res = round(float(z["map_resolution"]), 6)
    return P.Config(device=device, voxel_size_m=res, num_nei_cells=int(z["num_nei_cells"]),
                    search_alpha=float(z["search_alpha"]), query_nn_k=int(z["nn_k"]),
                    weighted_first=bool(z["weighted_first"]), buffer_size=int(z["map_buffer_size"]),
                    local_map_radius=15.0, query_backend=backend)


def neural_points_from_fixture(z, device="cuda", orientations=None, after_pgo=False, backend="auto"):
    cfg = config_from_fixture(z, device, backend)
    nm = P.NeuralPoints(cfg)
    t = lambda a, dt=None: torch.as_tensor(np.ascontiguousarray(a), device=device, dtype=dt)  # noqa: E731
    nm.diff_travel_dist_local = float(z["map_diff_travel_dist_local"])
    nm.neural_points = t(z["map_neural_points"], torch.float32)
    ori = z["map_point_orientations"] if orientations is None else orientations
    nm.point_orientations = t(ori, torch.float32)
    nm.geo_features = t(z["map_geo_features"], torch.float32)
    nm.point_ts_create = t(z["map_point_ts_create"], torch.int64)
    nm.point_ts_update = t(z["map_point_ts_update"], torch.int64)
    nm.point_certainties = t(z["map_point_certainties"], torch.float32)
    nm.travel_dist = t(z["map_travel_dist"], torch.float32)
    table = torch.full((nm.buffer_size,), -1, dtype=torch.int32, device=device)
    table[t(z["map_table_slots"], torch.int64)] = t(z["map_table_vals"], torch.int32)
    nm.buffer_pt_index = table
    nm.cur_ts = int(z["map_cur_ts"])
    # local map exactly as the reference left it
    mask = t(z["map_local_mask"], torch.bool)
    nm.local_mask = mask
    nm.global2local = t(z["map_global2local"], torch.int64)
    nm.local_neural_points = nm.neural_points[mask[:-1]]
    nm.local_point_orientations = nm.point_orientations[mask[:-1]]
    nm.local_point_certainties = nm.point_certainties[mask[:-1]]
    nm.local_point_ts_update = nm.point_ts_update[mask[:-1]]
    nm.local_geo_features = torch.nn.Parameter(nm.geo_features[mask])
    nm.after_pgo = after_pgo
    return nm


def decoder_from_fixture(z, cfg):
    dec = P.Decoder(cfg, 64, 1, 1)
    with torch.no_grad():
        dec.layers[0].weight.copy_(torch.as_tensor(z["dec_W1"]))
        dec.layers[0].bias.copy_(torch.as_tensor(z["dec_b1"]))
        dec.lout.weight.copy_(torch.as_tensor(z["dec_W2"]))
        dec.lout.bias.copy_(torch.as_tensor(z["dec_b2"]))
    assert abs(dec.sdf_scale - float(z["dec_sdf_scale"])) < 1e-7
    return dec


def oracle_state(nm) -> O.MapState:
    """Snapshot of a drop-in NeuralPoints as an oracle MapState (int64 table)."""
    c = lambda t: None if t is None else t.detach().cpu().numpy()  # noqa: E731
    table = c(nm.buffer_pt_index).astype(np.int64)
    st = O.MapState(resolution=nm.resolution, buffer_size=nm.buffer_size, table=table,
                    points=c(nm.neural_points), orientations=c(nm.point_orientations),
                    geo_features=c(nm.geo_features), ts_create=c(nm.point_ts_create),
                    ts_update=c(nm.point_ts_update), certainties=c(nm.point_certainties),
                    travel_dist=c(nm.travel_dist), cur_ts=int(nm.cur_ts),
                    diff_travel_dist_local=nm.diff_travel_dist_local, local_mask=c(nm.local_mask),
                    global2local=c(nm.global2local), local_points=c(nm.local_neural_points),
                    local_orientations=c(nm.local_point_orientations), local_features=c(nm.local_geo_features),
                    local_certainties=c(nm.local_point_certainties), local_ts_update=c(nm.local_point_ts_update),
                    after_pgo=nm.after_pgo)
    return st


def oracle_mlp(dec) -> O.MLP:
    c = lambda t: t.detach().cpu().numpy().astype(np.float32)  # noqa: E731
    return O.MLP(c(dec.layers[0].weight), c(dec.layers[0].bias), c(dec.lout.weight), c(dec.lout.bias),
                 float(dec.sdf_scale))


from pin_slam_amd.synthetic import surface_map, surface_queries  # noqa: E402,F401
