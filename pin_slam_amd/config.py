"""Hot-path configuration knobs with the reference defaults (utils/config.py:13-324).

The drop-in classes accept the reference's own ``utils.config.Config`` (or any
object with these attribute names); this class exists so the engine, its tests
and bench.py run without the reference tree.  Derived values follow
utils/config.py:568-574.
"""
import torch


class Config:
    def __init__(self, **overrides):
        self.device = "cuda"
        self.dtype = torch.float32
        self.silence = True
        self.seed = 42
        # neural points (utils/config.py:89-137)
        self.weighted_first = True
        self.layer_norm_on = False
        self.voxel_size_m = 0.3
        self.num_nei_cells = 2
        self.query_nn_k = 6
        self.use_mid_ts = False
        self.search_alpha = 0.2
        self.buffer_size = int(5e7)
        self.feature_dim = 8
        self.feature_std = 0.0
        self.diff_ts_local = 400.0
        self.local_map_travel_dist_ratio = 5.0
        self.local_map_radius = 50.0
        self.use_gaussian_pe = False
        self.pos_encoding_band = 0
        self.pos_input_dim = 3
        self.color_on = False
        self.semantic_on = False
        # sampler + data pool (:139-154, :205-207)
        self.surface_sample_n = 3
        self.free_sample_begin_ratio = 0.3
        self.free_sample_end_dist_m = 1.0
        self.free_front_n = 2
        self.free_behind_n = 1
        self.dist_weight_on = True
        self.dist_weight_scale = 0.8
        self.behind_dropoff_on = False
        self.window_radius = 50.0
        self.pool_capacity = int(1e7)
        self.bs_new_sample = 2048
        self.new_certainty_thre = 1.0
        self.pool_filter_freq = 10
        self.new_sample_ratio_thre = 0.01
        self.adaptive_mode = False
        self.from_sample_points = True
        self.from_all_samples = False
        self.map_surface_ratio = 0.5
        self.prune_map_on = False
        self.max_prune_certainty = 2.0
        self.dynamic_certainty_thre = 4.0
        self.dynamic_sdf_ratio_thre = 1.5
        self.pgo_on = False
        self.track_on = False
        self.color_channel = 0
        # decoder (:179-198)
        self.mlp_bias_on = True
        self.geo_mlp_level = 1
        self.geo_mlp_hidden_dim = 64
        self.main_loss_type = "bce"
        self.sigma_sigmoid_m = 0.1
        self.logistic_gaussian_ratio = 0.55
        self.loss_weight_on = False
        # mapper (:214-247)
        self.numerical_grad = True
        self.gradient_decimation = 10
        self.num_grad_step_ratio = 0.2
        self.ekional_loss_on = True
        self.ekional_add_to = "all"
        self.weight_e = 0.5
        self.iters = 15
        self.bs = 16384
        self.lr = 0.01
        self.weight_decay = 0.0
        self.adam_eps = 1e-15
        self.opt_adam = True
        # tracker (:157-174)
        self.surface_sample_range_m = 0.25
        self.reg_min_grad_norm = 0.5
        self.reg_max_grad_norm = 2.0
        self.max_sdf_ratio = 5.0
        self.max_sdf_std_ratio = 1.0
        self.reg_dist_div_grad_norm = False
        self.reg_GM_dist_m = 0.5
        self.reg_GM_grad = 0.2
        self.reg_lm_lambda = 1e-4
        self.reg_iter_n = 50
        self.reg_term_thre_deg = 0.01
        self.reg_term_thre_m = 0.0005
        self.eigenvalue_check = True
        self.photometric_loss_on = False
        # frame loop / dataset (pin_slam.py, dataset/slam_dataset.py; utils/config.py:45-67, :157-176,
        # :190, :235-241, :382, :483)
        self.deskew = False
        self.min_range = 2.5
        self.min_z = -4.0
        self.max_z = 60.0
        self.uniform_motion_on = True
        self.stop_frame_thre = 20
        self.freeze_after_frame = 40
        self.init_iter_ratio = 40
        self.mapping_freq_frame = 1
        # mesher (:296-308)
        self.mc_res_m = 0.1
        self.mesh_min_nn = 8
        self.infer_bs = 4096
        self.max_range = 60.0
        for k, v in overrides.items():
            setattr(self, k, v)
        if "infer_bs" not in overrides:
            self.infer_bs = self.bs * 64            # utils/config.py:569
        if "local_map_radius" not in overrides:
            self.local_map_radius = self.max_range + 2.0  # utils/config.py:574
        if "window_radius" not in overrides:
            self.window_radius = max(self.max_range, 6.0)  # utils/config.py:572
        if "vox_down_m" not in overrides:
            self.vox_down_m = self.max_range * 1e-3        # utils/config.py:382
        if "source_vox_down_m" not in overrides:
            self.source_vox_down_m = self.vox_down_m * 10  # utils/config.py:483
