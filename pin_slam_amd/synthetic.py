"""Synthetic workloads of SURVEY.md 8(d) (the KITTI example data is not available offline).

Map: one neural point per ``res`` voxel column on z = 0.5 sin(x/7) cos(y/5) + 0.15 over
an n x n grid, xy = (i + 0.5) * res; features ~ N(0, 0.05^2) (the reference default
feature_std = 0 would make the benchmark degenerate); decoder = nn.Linear default init
under torch.manual_seed(seed).  Queries: random map points + N(0, sigma^2) per axis.

Sequence (BASELINE configs[0], the plumbing run): a street of box buildings, cars and poles,
ray-cast by a 64-beam x 1024-column spinning lidar along an accelerating trajectory, and
``FrameLoop``, pin_slam.py's per-frame order (:96-257) over the drop-in classes with the
dataset's pose bookkeeping (dataset/slam_dataset.py:260-430) restated.
"""
import numpy as np
import torch

from .config import Config
from .decoder import Decoder
from .neural_points import NeuralPoints


def surface_points(n_side, res=0.3):
    i = torch.arange(n_side, dtype=torch.float64)
    x, y = torch.meshgrid((i + 0.5) * res, (i + 0.5) * res, indexing="ij")
    x, y = x.reshape(-1), y.reshape(-1)
    z = 0.5 * torch.sin(x / 7.0) * torch.cos(y / 5.0) + 0.15
    return torch.stack([x, y, z], 1).to(torch.float32)


def surface_map(n_side, res=0.3, seed=42, device="cuda", buffer_size=int(5e7), nn_k=8, weighted_first=True,
                feature_std=0.05, num_nei_cells=2, search_alpha=0.2, **cfg_kw):
    """Returns (NeuralPoints with the whole map local, Decoder, host points [M,3])."""
    return points_map(surface_points(n_side, res), res, seed, device, buffer_size, nn_k, weighted_first,
                      feature_std, num_nei_cells, search_alpha, **cfg_kw)


def points_map(pts, res=0.3, seed=42, device="cuda", buffer_size=int(5e7), nn_k=8, weighted_first=True,
               feature_std=0.05, num_nei_cells=2, search_alpha=0.2, **cfg_kw):
    """surface_map over the given host points [M,3] (random features and certainties)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    pts = torch.as_tensor(pts, dtype=torch.float32)
    cfg = Config(device=device, voxel_size_m=res, buffer_size=buffer_size, query_nn_k=nn_k,
                 weighted_first=weighted_first, local_map_radius=1e9, num_nei_cells=num_nei_cells,
                 search_alpha=search_alpha, **cfg_kw)
    nm = NeuralPoints(cfg)
    M = pts.shape[0]
    nm.neural_points = pts.to(device)
    quat = torch.zeros(M, 4, device=device)
    quat[:, 0] = 1.0
    nm.point_orientations = quat
    nm.point_ts_create = torch.zeros(M, dtype=torch.int64, device=device)
    nm.point_ts_update = torch.zeros(M, dtype=torch.int64, device=device)
    feats = torch.randn(M + 1, 8, generator=g) * feature_std
    feats[-1] = 0
    nm.geo_features = feats.to(device)
    nm.point_certainties = (torch.rand(M, generator=g) * 10).to(device)
    nm.travel_dist = torch.zeros(1, device=device)
    nm.rebuild_hash()
    nm.reset_local_map(torch.zeros(3, device=device), torch.eye(3, device=device), 0)
    torch.manual_seed(seed)
    dec = Decoder(cfg, 64, 1, 1)
    return nm, dec, pts


def surface_scan(cx, cy, radius, n, seed=0, sigma=0.02, device="cuda"):
    """A lidar-like frame: n points area-uniform in a disk of ``radius`` around (cx, cy) on the
    surface, z noise N(0, sigma^2).  Returns [n,3] f32 on ``device``."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    r = radius * torch.sqrt(torch.rand(n, generator=g, dtype=torch.float64))
    a = 2 * torch.pi * torch.rand(n, generator=g, dtype=torch.float64)
    x, y = cx + r * torch.cos(a), cy + r * torch.sin(a)
    z = 0.5 * torch.sin(x / 7.0) * torch.cos(y / 5.0) + 0.15 + sigma * torch.randn(n, generator=g, dtype=torch.float64)
    return torch.stack([x, y, z], 1).to(torch.float32).to(device)


def surface_queries(pts, n, seed=7, sigma=0.25, device="cuda"):
    g = torch.Generator(device="cpu").manual_seed(seed)
    idx = torch.randint(0, pts.shape[0], (n,), generator=g)
    q = pts[idx] + torch.randn(n, 3, generator=g) * sigma
    return q.to(device)


def surface_pool(pts, n, seed=11, sigma=0.25, device="cuda"):
    """Mapper training pool: map points offset along z by
    N(0, sigma^2), label = -offset, frame ts 0.  Returns (coord [n,3], label [n], ts [n])."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    idx = torch.randint(0, pts.shape[0], (n,), generator=g)
    off = torch.randn(n, generator=g) * sigma
    coord = pts[idx].clone()
    coord[:, 2] += off
    return coord.to(device), (-off).to(device), torch.zeros(n, dtype=torch.int64, device=device)


def train_surface(nm, dec, pts, iters=300, bs=16384, seed=3, pool=1 << 20):
    """Fit the map + decoder to the synthetic surface with the fused Mapper (sdf label = -z offset),
    so that SDF gradients are meaningful (tracker workloads).  Returns the last loss."""
    from .mapper import Mapper
    cfg = nm.config
    old_bs = cfg.bs
    cfg.bs = bs
    for p in dec.parameters():
        p.requires_grad_(True)
    coord, label, ts = surface_pool(pts, pool, seed=seed, device=nm.neural_points.device)
    mapper = Mapper(cfg, None, nm, dec)
    mapper.set_pool(coord, label, ts)
    torch.manual_seed(seed)
    mapper.mapping(iters)
    cfg.bs = old_bs
    nm.reset_local_map(torch.zeros(3, device=nm.neural_points.device),
                       torch.eye(3, device=nm.neural_points.device), 0)
    return float(mapper.last_loss)


# ------------------------------------------------------------------ the street sequence
SLAM_SENSOR_H = 1.73
Q_SCALE = 512.0   # sensor-frame points stored as int16 multiples of 2^-9 m (|coord| < 64 m)


def street_scene(rng):
    """Boxes (buildings, cars, a wall) and vertical cylinders (poles / trunks) on a ground plane,
    in the frame of the first sensor pose (ground at z = -1.73)."""
    g = -SLAM_SENSOR_H
    boxes = []
    x = -40.0
    while x < 70.0:       # two rows of buildings along the street
        w = rng.uniform(6.0, 14.0)
        for side in (-1.0, 1.0):
            y0 = side * rng.uniform(9.0, 12.0)
            d = rng.uniform(6.0, 12.0)
            ylo, yhi = (y0, y0 + d) if side > 0 else (y0 - d, y0)
            boxes.append((x, x + w, ylo, yhi, g, g + rng.uniform(5.0, 16.0)))
        x += w + rng.uniform(2.0, 6.0)
    for _ in range(10):   # parked cars
        cx = rng.uniform(-30.0, 60.0)
        cy = rng.choice([-1.0, 1.0]) * rng.uniform(4.5, 6.5)
        boxes.append((cx, cx + 4.2, cy - 0.9, cy + 0.9, g, g + 1.5))
    boxes.append((75.0, 76.0, -30.0, 30.0, g, g + 4.0))    # a wall across the street's end
    cyls = [(rng.uniform(-30.0, 60.0), rng.choice([-1.0, 1.0]) * rng.uniform(3.2, 7.5), rng.uniform(0.15, 0.45),
             g, g + rng.uniform(3.0, 8.0)) for _ in range(24)]
    return np.asarray(boxes), np.asarray(cyls), g


def long_street_scene(rng, length=200.0):
    """street_scene along a longer street (buildings from x = -40 to `length`, cars and poles
    spread over it, the wall at length + 5) for sequences of ~100 frames (long_slam_poses)."""
    g = -SLAM_SENSOR_H
    boxes = []
    x = -40.0
    while x < length:
        w = rng.uniform(6.0, 14.0)
        for side in (-1.0, 1.0):
            y0 = side * rng.uniform(9.0, 12.0)
            d = rng.uniform(6.0, 12.0)
            ylo, yhi = (y0, y0 + d) if side > 0 else (y0 - d, y0)
            boxes.append((x, x + w, ylo, yhi, g, g + rng.uniform(5.0, 16.0)))
        x += w + rng.uniform(2.0, 6.0)
    n_cars = int(length / 9)
    for _ in range(n_cars):
        cx = rng.uniform(-30.0, length - 10.0)
        cy = rng.choice([-1.0, 1.0]) * rng.uniform(4.5, 6.5)
        boxes.append((cx, cx + 4.2, cy - 0.9, cy + 0.9, g, g + 1.5))
    boxes.append((length + 5.0, length + 6.0, -30.0, 30.0, g, g + 4.0))
    cyls = [(rng.uniform(-30.0, length - 10.0), rng.choice([-1.0, 1.0]) * rng.uniform(3.2, 7.5),
             rng.uniform(0.15, 0.45), g, g + rng.uniform(3.0, 8.0)) for _ in range(int(length / 4))]
    return np.asarray(boxes), np.asarray(cyls), g


def long_slam_poses(frames, speed=1.2, ramp=10):
    """Sensor poses for long sequences: the speed ramps up over `ramp` frames to `speed` m/frame
    (KITTI-like at 10 Hz) and stays there, with a +-2.5 deg yaw and 0.15 m sway oscillation."""
    out = []
    x = 0.0
    for k in range(frames):
        if k > 0:
            x += speed * min(1.0, (k + 1) / ramp)
        yaw = np.deg2rad(2.5 * np.sin(0.11 * k) + 0.15 * np.sin(0.9 * k))
        T = np.eye(4)
        T[:3, :3] = [[np.cos(yaw), -np.sin(yaw), 0.0], [np.sin(yaw), np.cos(yaw), 0.0], [0.0, 0.0, 1.0]]
        T[:3, 3] = [x, 0.15 * np.sin(0.23 * k) + 0.08 * np.sin(0.7 * k), 0.005 * k]
        out.append(T)
    return out


def sequence_scene(kind, rng, frames):
    """(scene, poses) of a SLAM sequence fixture: "street" (street_scene + slam_poses, the 30-frame
    fixture) or "long" (long_street_scene + long_slam_poses, ~100 frames)."""
    if kind == "long":
        poses = long_slam_poses(frames)
        return long_street_scene(rng, length=float(poses[-1][0, 3]) + 60.0), poses
    return street_scene(rng), slam_poses(frames)


def lidar_scan(pose, scene, rng, beams=64, cols=1024, noise=0.01):
    """A 64-beam spinning lidar at `pose` (4x4, f64) ray-cast against the scene; returns the hits in
    the sensor frame, ranges in [3, 59.5] m (so the reference's crop_frame is a no-op), quantised
    to multiples of 2^-9 m (int16 storage, exact in float32)."""
    boxes, cyls, ground = scene
    el = np.deg2rad(np.linspace(-24.8, 2.0, beams))
    az = np.linspace(-np.pi, np.pi, cols, endpoint=False)
    E, A = np.meshgrid(el, az, indexing="ij")
    ds = np.stack([np.cos(E) * np.cos(A), np.cos(E) * np.sin(A), np.sin(E)], -1).reshape(-1, 3)
    R, o = pose[:3, :3], pose[:3, 3]
    d = ds @ R.T
    t = np.full(d.shape[0], np.inf)
    with np.errstate(divide="ignore", invalid="ignore"):
        tg = (ground - o[2]) / d[:, 2]
        t = np.where((d[:, 2] < 0) & (tg > 0), np.minimum(t, tg), t)
        for (x0, x1, y0, y1, z0, z1) in boxes:
            lo = (np.array([x0, y0, z0]) - o) / d
            hi = (np.array([x1, y1, z1]) - o) / d
            tn = np.minimum(lo, hi).max(1)
            tf = np.maximum(lo, hi).min(1)
            hit = (tn <= tf) & (tn > 0)
            t = np.where(hit, np.minimum(t, tn), t)
        for (cx, cy, r, z0, z1) in cyls:
            px, py = o[0] - cx, o[1] - cy
            a = d[:, 0] ** 2 + d[:, 1] ** 2
            b = 2 * (px * d[:, 0] + py * d[:, 1])
            cc = px * px + py * py - r * r
            disc = b * b - 4 * a * cc
            tc = (-b - np.sqrt(np.maximum(disc, 0))) / (2 * a)
            zc = o[2] + tc * d[:, 2]
            hit = (disc > 0) & (tc > 0) & (zc > z0) & (zc < z1)
            t = np.where(hit, np.minimum(t, tc), t)
    t = t + rng.normal(0.0, noise, t.shape)
    keep = np.isfinite(t) & (t > 3.0) & (t < 59.5)
    p = ds[keep] * t[keep, None]
    q = np.round(p * Q_SCALE)
    assert np.abs(q).max() < 32767
    return q.astype(np.int16)


def slam_poses(frames):
    """Sensor poses in the first pose's frame: accelerating along the street (0.22 m in the first
    frame, ~1.6 m per frame by frame 11: the first guess is the identity, later ones the
    constant-velocity model, off by the 0.14 m/frame^2 acceleration), a slow yaw and sway."""
    out = []
    for k in range(frames):
        yaw = np.deg2rad(0.6 * k + 0.15 * np.sin(0.9 * k))
        T = np.eye(4)
        T[:3, :3] = [[np.cos(yaw), -np.sin(yaw), 0.0], [np.sin(yaw), np.cos(yaw), 0.0], [0.0, 0.0, 1.0]]
        T[:3, 3] = [0.15 * k + 0.07 * k * k, 0.08 * np.sin(0.7 * k), 0.01 * k]
        out.append(T)
    return out



class FrameLoop:
    """pin_slam.py:96-257 on the drop-in classes for scans already in memory: read (identity pose,
    no pose file), voxel down-sample + crop, constant-velocity guess, source cloud, tracking,
    update_odom_pose, travel distance, process_frame, decoder freeze, mapping(iters) -- the
    dataset bookkeeping of dataset/slam_dataset.py:260-430 restated (deskew off).  ``draws``
    (optional callable n -> (randn, rand, rand)) replays the sampler's draws."""

    def __init__(self, cfg, nm, dec, tracker, mapper, build_index=False):
        self.config, self.nm, self.dec, self.tracker, self.mapper = cfg, nm, dec, tracker, mapper
        # build_index: build the query index of the updated map (occupancy grid + compact records)
        # as a part of its own before tracking, instead of inside the tracker's first query
        self.build_index = build_index
        self.dev = nm.neural_points.device
        self.odom_poses, self.travel_dist = [], []
        self.processed_frame = 0
        self.lose_track = False
        self.last_pose_ref = np.eye(4)
        self.last_odom_tran = np.eye(4)
        self.cur_pose_ref = np.eye(4)
        self.stop_count = 0
        self.stop_status = False
        self.gt_pose_provided = False
        mapper.dataset = self

    def _clouds(self, pts, want_source):
        """The scan's own preprocessing (slam_dataset.py:260-345): voxel down-sample, crop and --
        after frame 0 -- the registration's source down-sample.  A function of the scan alone."""
        from .neural_points import voxel_down_sample
        c = self.config
        cloud = pts[voxel_down_sample(pts, c.vox_down_m)]                 # slam_dataset.py:286
        dist = torch.norm(cloud, dim=1)                                    # crop_frame, :827-834
        keep = (dist > c.min_range) & (dist < c.max_range) & (cloud[:, 2] > c.min_z) & (cloud[:, 2] < c.max_z)
        cloud = cloud[keep]
        src = cloud[voxel_down_sample(cloud, c.source_vox_down_m)] if want_source else None
        return cloud, src

    def prefetch(self, pts, ready=None):
        """Preprocess the NEXT scan on a side stream while the device works through this frame's
        mapping (its host syncs then wait for the side stream only): the scan's preprocessing does
        not depend on the map, so read_and_preprocess of that scan only picks the result up.  The
        outputs are the same tensors, bitwise, as preprocessing it in turn."""
        if self.__dict__.get("_side") is None:
            self._side = torch.cuda.Stream(device=self.dev)
        main = torch.cuda.current_stream(self.dev)
        # the scan was produced before ``ready`` (an event of the main stream recorded when the
        # scan was handed over): waiting for it, and not for everything queued since (this
        # frame's mapping), keeps the side stream beside the mapping kernels
        if ready is not None:
            self._side.wait_event(ready)
        else:
            self._side.wait_stream(main)
        with torch.cuda.stream(self._side):
            cloud, src = self._clouds(pts, True)
            done = torch.cuda.Event()
            done.record(self._side)
        for t in (cloud, src):          # allocated on the side stream, read on the main one
            if t is not None:
                t.record_stream(main)
        self._prefetched = (pts, cloud, src, done)

    def _h2d(self, a, dtype):
        """A small host array on the device without a blocking copy: staged in pinned memory (the
        caching host allocator keeps it until the stream-ordered copy has run)."""
        return torch.from_numpy(np.ascontiguousarray(a)).to(dtype).pin_memory().to(self.dev, non_blocking=True)

    def read_and_preprocess(self, pts):
        c = self.config
        self.cur_pose_ref = np.eye(4)
        self.cur_pose_torch = self._h2d(self.cur_pose_ref, torch.float32)
        pre = self.__dict__.pop("_prefetched", None)
        if pre is not None and pre[0] is pts:
            torch.cuda.current_stream(self.dev).wait_event(pre[3])
            cloud, src = pre[1], pre[2]
        else:
            cloud, src = self._clouds(pts, self.processed_frame > 0)
        self.cur_point_cloud_torch = cloud
        self.cur_source_points = None
        if self.processed_frame == 0:
            self.odom_poses.append(self.cur_pose_ref)
            self.travel_dist.append(0.0)
            self.last_pose_ref = self.cur_pose_ref
        else:                                                              # :320-339
            guess = self.last_pose_ref @ self.last_odom_tran if (c.uniform_motion_on and not self.lose_track) \
                else self.last_pose_ref
            self.cur_pose_guess_torch = self._h2d(guess, torch.float64)
            self.cur_source_points = src

    def update_odom_pose(self, cur_pose_torch):
        """dataset/slam_dataset.py:376-430."""
        c = self.config
        self.cur_pose_torch = cur_pose_torch.detach()
        self.cur_pose_ref = self.cur_pose_torch.cpu().numpy()
        self.last_odom_tran = np.linalg.inv(self.last_pose_ref) @ self.cur_pose_ref
        rot_close = np.all(np.abs(self.last_odom_tran[:3, :3] - np.eye(3)) < 1e-3)
        tran_close = np.all(self.last_odom_tran[:3, 3] < c.voxel_size_m * 0.1)
        self.stop_count = self.stop_count + 1 if (rot_close and tran_close) else 0
        self.stop_status = self.stop_count > c.stop_frame_thre
        self.odom_poses.append(self.odom_poses[-1] @ self.last_odom_tran)
        step = np.linalg.norm(self.last_odom_tran[:3, 3])
        if step > c.surface_sample_range_m * 40.0:
            self.lose_track = True
        self.travel_dist.append(self.travel_dist[-1] + step)
        self.last_pose_ref = self.cur_pose_ref

    def frame(self, pts, draws=None, timer=None, next_pts=None):
        """One frame of the loop; timer(name) (optional) is called at each part's end.  next_pts
        (optional): the next scan, preprocessed on a side stream while this frame's mapping runs
        (prefetch); its mapping() leaves the device-side batch check to the next call
        (Mapper.defer_checks), so the host is free for that while the device maps."""
        c, nm, mapper = self.config, self.nm, self.mapper
        mark = timer or (lambda name: None)
        used = self.processed_frame
        handed = None
        if next_pts is not None:   # everything that produced next_pts is queued before this point
            handed = torch.cuda.Event()
            handed.record()
        self.read_and_preprocess(pts)
        mark("preprocess")
        if self.build_index and used > 0 and nm.backend() == "grid":
            nm.grid_view("local", True)
            mark("index")
        valid = True
        if used > 0:
            T, _, _, valid = self.tracker.tracking(self.cur_source_points, self.cur_pose_guess_torch, None, None)
            self.lose_track = not valid
            mapper.lose_track = not valid
            self.update_odom_pose(T)
        mark("tracking")
        nm.travel_dist = self._h2d(np.array(self.travel_dist), torch.float32)
        if not mapper.lose_track and not self.stop_status:
            d = draws(self.cur_point_cloud_torch.shape[0]) if draws is not None else None
            mapper.process_frame(self.cur_point_cloud_torch, None, self.cur_pose_torch, used, False, draws=d)
        else:
            nm.reset_local_map(self.cur_pose_torch[:3, 3], None, used)
        mark("process_frame")
        iters = c.iters * c.init_iter_ratio if used == 0 else c.iters
        if used == c.freeze_after_frame:
            for p in self.dec.parameters():
                p.requires_grad_(False)
        if used % c.mapping_freq_frame == 0:
            mapper.defer_checks = next_pts is not None
            mapper.mapping(iters)
        if next_pts is not None:
            self.prefetch(next_pts, handed)
        mark("mapping")
        self.processed_frame += 1
        return valid


# KITTI-style settings (config/lidar_slam/run_kitti.yaml) for the configs[2] registration workload
KITTI_CFG = dict(voxel_size_m=0.4, query_nn_k=6, search_alpha=0.5, weighted_first=False, surface_sample_range_m=0.25,
                 surface_sample_n=4, free_front_n=2, sigma_sigmoid_m=0.08, loss_weight_on=True, dist_weight_scale=0.8,
                 bs_new_sample=2000, pool_capacity=int(2e7), freeze_after_frame=30, reg_iter_n=100, reg_GM_grad=0.1,
                 reg_GM_dist_m=0.2, max_range=80.0, min_range=3.0, vox_down_m=0.08, min_z=-3.5,
                 source_vox_down_m=0.8, track_on=True)


def street_map(frames=12, device="cuda", seed=21, cfg_overrides=None, deterministic=True):
    """A neural-point map of the synthetic street built by PIN-SLAM's mapping steps with the
    ground-truth poses (pin_slam.py:161-257 with tracking replaced by the known pose, i.e. the
    reference's mapping-only mode): per frame voxel down-sample + crop, process_frame (sampling,
    map update, pool), mapping(iters; 40 x on frame 0) with the decoder training.  KITTI settings
    (KITTI_CFG) unless overridden.  Returns (nm, dec, cfg, scene, poses, rng); the map is centred
    on the last pose's local map.  deterministic: the mapper's deterministic mode, so the same
    arguments give the same map bitwise (the draws come from torch's seeded generators)."""
    from .mapper import Mapper
    from .neural_points import voxel_down_sample
    kw = dict(KITTI_CFG)
    kw.update(cfg_overrides or {})
    cfg = Config(device=device, **kw)
    rng = np.random.default_rng(seed)
    scene = street_scene(rng)
    poses = slam_poses(frames + 1)
    nm = NeuralPoints(cfg)
    torch.manual_seed(42)
    dec = Decoder(cfg, cfg.geo_mlp_hidden_dim, cfg.geo_mlp_level, 1).to(device)
    mapper = Mapper(cfg, None, nm, dec, deterministic=deterministic)
    travel = [0.0]
    for k in range(frames):
        if k > 0:
            travel.append(travel[-1] + float(np.linalg.norm(poses[k][:3, 3] - poses[k - 1][:3, 3])))
        pts = torch.from_numpy(lidar_scan(poses[k], scene, rng).astype(np.float32) / np.float32(Q_SCALE)).to(device)
        cloud = pts[voxel_down_sample(pts, cfg.vox_down_m)]
        dist = torch.norm(cloud, dim=1)
        cloud = cloud[(dist > cfg.min_range) & (dist < cfg.max_range) & (cloud[:, 2] > cfg.min_z) &
                      (cloud[:, 2] < cfg.max_z)]
        pose = torch.tensor(poses[k], dtype=torch.float32, device=device)
        nm.travel_dist = torch.tensor(np.array(travel), dtype=torch.float32, device=device)
        mapper.process_frame(cloud, None, pose, k, False)
        if k == cfg.freeze_after_frame:
            for p in dec.parameters():
                p.requires_grad_(False)
        mapper.mapping(cfg.iters * cfg.init_iter_ratio if k == 0 else cfg.iters)
    return nm, dec, cfg, scene, poses, rng


def perturb_pose(T, dx=0.2, yaw_deg=0.5):
    """T (4x4 f64) moved by dx metres along its x axis and rotated by yaw_deg about z."""
    a = np.deg2rad(yaw_deg)
    D = np.eye(4)
    D[:3, :3] = [[np.cos(a), -np.sin(a), 0.0], [np.sin(a), np.cos(a), 0.0], [0.0, 0.0, 1.0]]
    D[0, 3] = dx
    return T @ D
