"""ctypes binding of libpin_slam_amd.so (the C ABI declared in include/pin_slam_amd.h).

The library is REQUIRED: there is no CPU or eager-PyTorch fallback for the hot
path.  If the shared object is missing or a call fails, this module raises.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# PIN_LIB overrides the library path (experiment variants built by tools/variants.py)
LIB_PATH = os.environ.get("PIN_LIB") or os.path.join(_HERE, "libpin_slam_amd.so")

PIN_OK = 0
PIN_TRAIN_ROWS = 1   # PinTrainCfg.flags: coord holds every row of the iteration
PIN_TRAIN_DX = 2     # PinTrainCfg.flags: forward saves s dsdf/dx (matrix-core decoder), backward applies it
PIN_TRAIN_EIK = 4    # PinTrainCfg.flags: analytic-gradient eikonal (double backward in closed form)
PIN_TRAIN_PAIR = 8   # PinTrainCfg.flags: two lanes per row in the forward (small batches)
PIN_RECORD_UNFAITHFUL = 1 << 30   # record id flag (pin_build_records)
PIN_QUERY_OUT_TILE = 1   # outputs in tile order (pin_query_sdf_grid_*_ex)
PIN_GRID_TABLE_TRUSTED = 1   # pin_grid_mark_ex: skip the table count
_ERRORS = {-1: "invalid argument", -2: "HIP launch/runtime failure", -3: "unsupported configuration"}

FEATURE_DIM = 8
MAX_NN_K = 8
HIDDEN_DIM = 64
RECORD_UNFAITHFUL = 1 << 30

c_void_p = ctypes.c_void_p
i32 = ctypes.c_int32
i64 = ctypes.c_int64
f32 = ctypes.c_float


class PinHash(ctypes.Structure):
    _fields_ = [("table", c_void_p), ("buffer_size", i64), ("resolution", f32), ("num_cells", i32),
                ("cells", c_void_p), ("max_valid_dist2", f32), ("reserved", i32)]


class PinPoints(ctypes.Structure):
    _fields_ = [("records", c_void_p), ("num_points", i64), ("features", c_void_p), ("positions", c_void_p),
                ("orientations", c_void_p), ("certainties", c_void_p), ("rows", i64), ("after_pgo", i32),
                ("reserved", i32), ("positions4", c_void_p)]


class PinGridDims(ctypes.Structure):
    _fields_ = [("ox", i64), ("oy", i64), ("oz", i64), ("nbx", i32), ("nby", i32), ("nbz", i32), ("reserved", i32)]


class PinSampleCfg(ctypes.Structure):
    _fields_ = [("surface_n", i32), ("front_n", i32), ("behind_n", i32), ("surface_range", f32), ("two_range", f32),
                ("front_min_ratio", f32), ("end_dist", f32), ("dist_weight_on", i32), ("dist_weight_base", f32),
                ("dist_weight_scale", f32), ("max_range", f32), ("behind_dropoff_on", i32), ("dropoff_max", f32),
                ("dropoff_diff", f32), ("pose", c_void_p)]


class PinGrid(ctypes.Structure):
    _fields_ = [("bricks", c_void_p), ("dims", PinGridDims), ("crec", c_void_p), ("cgid", c_void_p), ("n_occ", i64),
                ("offsets", c_void_p), ("resolution", f32), ("num_cells", i32), ("max_valid_dist2", f32),
                ("cfeat", c_void_p), ("ccert", c_void_p), ("fat", i32), ("window", i32), ("num_columns", i32)]


class PinRegParams(ctypes.Structure):
    _fields_ = [("min_nn_count", i32), ("min_grad_norm", f32), ("max_grad_norm", f32), ("max_sdf_std", f32),
                ("gm_dist", f32), ("gm_grad", f32), ("div_grad_norm", i32), ("q4_points", i32)]


class PinRegIter(ctypes.Structure):
    _fields_ = [("src", c_void_p), ("n", i64), ("labels", c_void_p), ("cur", c_void_p), ("q4", c_void_p),
                ("order_ws", c_void_p), ("sdf", c_void_p), ("grad", c_void_p), ("nn_count", c_void_p),
                ("sdf_std", c_void_p), ("reg_ws", c_void_p), ("acc_status_dt", c_void_p), ("host_out", c_void_p),
                ("nn_k", i32), ("weighted_first", i32), ("lm_lambda", ctypes.c_double), ("prm", PinRegParams)]


REG_NACC = 31
REG_NSTATUS = 8
REG_WORKSPACE_DOUBLES = 256 * REG_NACC + 8   # block partials + pin_reg_step's counter word


class PinMlp(ctypes.Structure):
    _fields_ = [("W1", c_void_p), ("b1", c_void_p), ("W2", c_void_p), ("b2", c_void_p), ("sdf_scale", f32),
                ("reserved", i32), ("packed", c_void_p)]


MLP_PACK_BYTES = 8288


class PinTrainCfg(ctypes.Structure):
    _fields_ = [("n_main", i64), ("n_stencil", i64), ("decimation", i32), ("nn_k", i32), ("weighted_first", i32),
                ("eps", f32), ("sigma", f32), ("weight_e", f32), ("grad_scale", f32), ("flags", i32),
                ("n_tail", i64), ("grad_scale_tail", f32), ("reserved", i32)]


class PinTrainState(ctypes.Structure):
    _fields_ = [("ids", c_void_p), ("weights", c_void_p), ("x", c_void_p), ("sdf", c_void_p),
                ("certainties", c_void_p), ("ts_update", c_void_p), ("order", c_void_p), ("sorted_rows", c_void_p),
                ("row_weight", c_void_p), ("eik_coef", c_void_p), ("eik_vec", c_void_p), ("row_ts", c_void_p),
                ("grad_replicas", c_void_p), ("replicas", i32), ("replica_mode", i32),
                ("grad_fixed", c_void_p), ("cert_fixed", c_void_p), ("fixed_shift", i32), ("cert_shift", i32)]


class PinAdamStep(ctypes.Structure):
    _fields_ = [("neg_step_size", f32), ("one_minus_beta1", f32), ("beta2", f32), ("one_minus_beta2", f32),
                ("bias_correction2_sqrt", f32), ("eps", f32), ("zero_grad", i32), ("grad_stride", i32)]


class PinMapArrays(ctypes.Structure):
    _fields_ = [("positions", c_void_p), ("orientations", c_void_p), ("ts_create", c_void_p), ("ts_update", c_void_p),
                ("certainties", c_void_p), ("features", c_void_p), ("count", i64), ("feature_dim", i32),
                ("reserved", i32)]


class PinRowArray(ctypes.Structure):
    _fields_ = [("src", c_void_p), ("dst", c_void_p), ("row_bytes", i64)]


ROW_ARRAYS_MAX = 8   # PIN_ROW_ARRAYS_MAX
MLP_GRAD_FIRST, MLP_GRAD_SECOND = 1, 2   # pin_mlp_backward flags

MLP_GRAD_SIZE = HIDDEN_DIM * (FEATURE_DIM + 3) + 2 * HIDDEN_DIM + 1
MLP_PART_FLOATS = 2 * HIDDEN_DIM * 16 + 16   # PIN_MLP_PART_FLOATS: per-block decoder-gradient partial

_P = ctypes.POINTER
# name -> (argtypes) ; every function returns int
_SIGS = {
    "pin_build_records": [c_void_p, i64, i32, c_void_p, c_void_p, c_void_p, i64, i64, f32, c_void_p, i64,
                          c_void_p, c_void_p],
    "pin_neighbor_cells": [c_void_p, i32, i64, c_void_p, c_void_p],
    "pin_hash_rebuild": [c_void_p, i64, f32, c_void_p, i64, c_void_p],
    "pin_radius_search": [_P(PinHash), _P(PinPoints), c_void_p, i64, c_void_p, c_void_p, c_void_p],
    "pin_query_sdf": [_P(PinHash), _P(PinPoints), _P(PinMlp), c_void_p, i64, i32, i32, i32, c_void_p, c_void_p,
                      c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_query_feature_fwd": [_P(PinHash), _P(PinPoints), c_void_p, i64, i32, i32, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_query_feature_bwd": [_P(PinPoints), c_void_p, i64, i32, i32, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_query_feature_bwd2": [_P(PinPoints), c_void_p, i64, i32, i32, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_train_scatter": [c_void_p, c_void_p, i64, i32, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_query_certainty": [_P(PinHash), _P(PinPoints), c_void_p, i64, c_void_p, c_void_p],
    "pin_reg_normal_eq": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, i64,
                          _P(PinRegParams), c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_cell_bounds": [c_void_p, i64, f32, c_void_p, c_void_p],
    "pin_reg_solve": [c_void_p, ctypes.c_double, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_reg_step": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, i64, _P(PinRegParams), c_void_p,
                     c_void_p, ctypes.c_double, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_transform_points": [c_void_p, i64, c_void_p, c_void_p, c_void_p],
    "pin_transform_points_sorted": [c_void_p, i64, c_void_p, c_void_p, c_void_p],
    "pin_reg_iteration": [_P(PinGrid), _P(PinHash), _P(PinPoints), _P(PinMlp), _P(PinRegIter), i32, c_void_p, c_void_p,
                          c_void_p],
    "pin_grid_mark": [c_void_p, i64, f32, c_void_p, i64, _P(PinGridDims), c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_grid_mark_ex": [c_void_p, i64, f32, c_void_p, i64, _P(PinGridDims), c_void_p, c_void_p, c_void_p, i32,
                         c_void_p],
    "pin_grid_fill": [c_void_p, i64, f32, c_void_p, i64, _P(PinGridDims), c_void_p, c_void_p, c_void_p, c_void_p,
                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_query_sdf_grid": [_P(PinGrid), _P(PinPoints), _P(PinMlp), c_void_p, i64, i32, i32, i32, c_void_p, c_void_p,
                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_mlp_pack": [_P(PinMlp), c_void_p, c_void_p],
    "pin_query_order": [_P(PinGrid), c_void_p, i64, c_void_p, c_void_p, c_void_p],
    "pin_query_sort": [_P(PinGrid), c_void_p, i64, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_query_sort_stable_workspace_bytes": [i64],
    "pin_query_sort_stable": [_P(PinGrid), c_void_p, i64, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_query_sdf_grid_tiled": [_P(PinGrid), _P(PinPoints), _P(PinMlp), c_void_p, i64, i32, i32, i32, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_query_sdf_grid_sorted": [_P(PinGrid), _P(PinPoints), _P(PinMlp), c_void_p, i64, i32, i32, i32, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_query_sdf_grid_tiled_ex": [_P(PinGrid), _P(PinPoints), _P(PinMlp), c_void_p, i64, i32, i32, i32, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, i32, c_void_p],
    "pin_query_sdf_grid_sorted_ex": [_P(PinGrid), _P(PinPoints), _P(PinMlp), c_void_p, i64, i32, i32, i32, c_void_p,
                                     c_void_p, c_void_p, c_void_p, c_void_p, i32, c_void_p],
    "pin_mc_workspace_bytes": [i64, i64, i64],
    "pin_mc_count": [c_void_p, c_void_p, i64, i64, i64, f32, c_void_p, c_void_p, c_void_p],
    "pin_mc_emit": [c_void_p, i64, i64, i64, f32, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_deskew": [c_void_p, i64, i64, c_void_p, c_void_p, c_void_p, f32, c_void_p],
    "pin_sample_rays": [c_void_p, i64, c_void_p, c_void_p, c_void_p, _P(PinSampleCfg), c_void_p, c_void_p, c_void_p,
                        c_void_p, c_void_p],
    "pin_query_feature_fwd_grid": [_P(PinGrid), _P(PinPoints), c_void_p, i64, i32, i32, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_train_rows": [c_void_p, _P(PinTrainCfg), c_void_p, c_void_p],
    "pin_train_gather": [c_void_p, c_void_p, c_void_p, c_void_p, i64, c_void_p, _P(PinTrainCfg), c_void_p, c_void_p,
                         c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_pool_pack": [c_void_p, c_void_p, c_void_p, c_void_p, i64, c_void_p, c_void_p],
    "pin_train_gather_packed": [c_void_p, i64, c_void_p, _P(PinTrainCfg), c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p],
    "pin_train_gather_packed_split": [c_void_p, i64, c_void_p, i64, c_void_p, i64, c_void_p, _P(PinTrainCfg), c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_train_gather_packed_draw": [c_void_p, i64, i64, c_void_p, i64, ctypes.c_uint64, ctypes.c_uint64,
                                     _P(PinTrainCfg), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_train_forward": [_P(PinHash), _P(PinGrid), _P(PinPoints), _P(PinMlp), c_void_p, c_void_p, _P(PinTrainCfg),
                          _P(PinTrainState), c_void_p],
    "pin_train_backward": [_P(PinPoints), _P(PinMlp), c_void_p, _P(PinTrainCfg), _P(PinTrainState), c_void_p,
                           c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_adam_step": [c_void_p, c_void_p, c_void_p, c_void_p, i64, _P(PinAdamStep), c_void_p],
    "pin_adam_rows": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, i64, _P(PinAdamStep), c_void_p],
    "pin_adam_step_train": [c_void_p, c_void_p, c_void_p, c_void_p, i64, c_void_p, i32, c_void_p, i32, _P(c_void_p),
                            _P(i64), i32, c_void_p, c_void_p, c_void_p, _P(PinMlp), c_void_p, _P(PinAdamStep), c_void_p],
    "pin_fixed_accumulate": [c_void_p, i32, i64, i32, i32, c_void_p, c_void_p],
    "pin_ref_sort_rows": [c_void_p, i32, i64, c_void_p, c_void_p],
    "pin_adam_segments": [_P(c_void_p), _P(i64), i32, c_void_p, c_void_p, c_void_p, _P(PinAdamStep), c_void_p],
    "pin_adam_step_segments": [c_void_p, c_void_p, c_void_p, c_void_p, i64, _P(c_void_p), _P(i64), i32, c_void_p,
                               c_void_p, c_void_p, _P(PinAdamStep), c_void_p],
    "pin_map_workspace_bytes": [i64],
    "pin_voxel_down_sample": [c_void_p, i64, f32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_map_insert": [c_void_p, c_void_p, i64, f32, c_void_p, i64, c_void_p, c_void_p, i64, c_void_p, i64, f32, f32,
                       c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_hash_assign": [c_void_p, c_void_p, i64, f32, c_void_p, i64, c_void_p, c_void_p],
    "pin_local_map": [_P(PinMapArrays), c_void_p, c_void_p, i32, i64, ctypes.c_double, f32, i32, i32, i64, i64,
                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_prune_rows": [_P(PinMapArrays), c_void_p, i64, f32, f32, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_mlp_forward": [_P(PinMlp), c_void_p, i64, c_void_p, c_void_p],
    "pin_mlp_backward_workspace_bytes": [i64],
    "pin_mlp_backward": [_P(PinMlp), c_void_p, i64, c_void_p, c_void_p, i32, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p],
    "pin_pool_window_workspace_bytes": [i64],
    "pin_pool_window": [c_void_p, i64, c_void_p, i32, ctypes.c_double, i64, c_void_p, c_void_p, c_void_p, c_void_p],
    "pin_gather_rows": [_P(PinRowArray), i32, c_void_p, i64, c_void_p],
    "pin_map_gather": [_P(PinMapArrays), c_void_p, i64, i32, _P(PinMapArrays), c_void_p],
    "pin_map_scatter": [_P(PinMapArrays), c_void_p, i64, i32, _P(PinMapArrays), c_void_p],
    "pin_map_adjust": [_P(PinMapArrays), c_void_p, i64, i32, c_void_p],
}
# functions whose return value is not a status code
_RESTYPES = {"pin_map_workspace_bytes": i64, "pin_mc_workspace_bytes": i64,
             "pin_query_sort_stable_workspace_bytes": i64, "pin_mlp_backward_workspace_bytes": i64,
             "pin_pool_window_workspace_bytes": i64}

_lib = None


def exported_symbols():
    return sorted(_SIGS)


def load():
    """Load the shared library (no GPU needed to load).  Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"pin_slam_amd: native library not built ({LIB_PATH}); run `python -m pin_slam_amd.build` "
                           "or __graft_entry__.build(). There is no fallback path.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    _lib = lib
    return lib


def call(name, *args):
    rc = getattr(load(), name)(*args)
    if rc != PIN_OK:
        raise RuntimeError(f"{name} failed: {_ERRORS.get(rc, rc)}")


def fn(name):
    """The bound entry point itself (hot loops: call it and pass its status to check)."""
    return getattr(load(), name)


def check(name, rc):
    if rc != PIN_OK:
        raise RuntimeError(f"{name} failed: {_ERRORS.get(rc, rc)}")


def map_workspace_bytes(n):
    b = load().pin_map_workspace_bytes(int(n))
    if b < 0:
        raise RuntimeError(f"pin_map_workspace_bytes failed: {_ERRORS.get(b, b)}")
    return b


def ptr(t):
    """Device pointer of a tensor (None -> NULL).  The tensor must be contiguous."""
    if t is None:
        return None
    if not t.is_contiguous():
        raise ValueError("pin_slam_amd: kernels need contiguous tensors")
    return c_void_p(t.data_ptr())


try:
    _raw_stream = torch._C._cuda_getCurrentRawStream   # no Stream object per call (~0.2 vs ~3 us)
except AttributeError:   # pragma: no cover
    _raw_stream = None


def stream(device=None):
    """The current HIP stream of ``device`` (default: the current device) as a c_void_p."""
    if _raw_stream is not None:
        if device is None:
            idx = torch.cuda.current_device()
        elif isinstance(device, int):
            idx = device
        else:
            idx = torch.device(device).index
            idx = torch.cuda.current_device() if idx is None else idx
        return c_void_p(_raw_stream(idx))
    return c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device(t):
    if not t.is_cuda:
        raise RuntimeError("pin_slam_amd: the HIP kernels need tensors on a ROCm device (got %s); the hot path has "
                           "no CPU implementation" % t.device)
