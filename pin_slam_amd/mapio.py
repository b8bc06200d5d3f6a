"""PIN map files (``model/pin_map.pth``) in the reference's on-disk format.

The reference writes a map with ``utils/tools.py:224-238`` (``save_implicit_map``)::

    torch.save({"neural_points": <model.neural_points.NeuralPoints, pickled nn.Module>,
                "geo_decoder": Decoder.state_dict(), ["color_decoder": ..., "sem_decoder": ...]},
               run_path/model/pin_map.pth)

and reads it back with a plain ``torch.load`` (``vis_pin_map.py:54-63``, ``utils/tools.py:257-259``).

``load_pin_map`` reads such a file WITHOUT executing anything from it: ``torch.load(...,
weights_only=True)`` with the reference's classes (``model.neural_points.NeuralPoints``, its
position encoders and ``utils.config.Config``) bound to inert record types here, so the
unpickler only rebuilds tensors and plain containers and hands each object's state dict to a
record.  The map state is then installed into this package's ``NeuralPoints`` (the hash table
narrowed to int32, local-map tensors kept), on the requested device.

``save_implicit_map`` writes the same structure from a ``pin_slam_amd.NeuralPoints``: the
pickle names the reference's classes, so the reference's own ``torch.load`` (with the
reference tree importable) rebuilds a real ``model.neural_points.NeuralPoints``.
"""
import collections
import os
import sys
import types

import numpy as np
import torch

from .config import Config
from .neural_points import NeuralPoints

_REF_NP = ("model.neural_points", "NeuralPoints")
_REF_CFG = ("utils.config", "Config")
_REF_ENCODERS = [("model.neural_points", "GaussianFourierFeatures"), ("model.neural_points", "PositionalEncoder")]

# NeuralPoints tensors / scalars carried by the file (model/neural_points.py:22-100)
_MAP_TENSORS = ["neural_points", "point_orientations", "geo_features", "color_features", "point_ts_create",
                "point_ts_update", "point_certainties", "local_neural_points", "local_point_orientations",
                "local_point_certainties", "local_point_ts_update", "local_mask", "global2local", "travel_dist",
                "est_poses", "local_orientation"]
_MAP_SCALARS = ["cur_ts", "max_ts", "after_pgo", "resolution", "buffer_size", "local_map_radius",
                "diff_travel_dist_local", "diff_ts_local", "temporal_local_map_on", "memory_footprint"]


class _Record:
    """Inert stand-in for a pickled reference object: keeps the unpickled state dict only."""

    def __setstate__(self, state):
        self.__dict__["_state"] = state if isinstance(state, dict) else {"_raw": state}

    @property
    def state(self):
        return self.__dict__.get("_state", {})


def _record_type(module, name):
    return type(name, (_Record,), {"__module__": "pin_slam_amd.mapio._ref", "__qualname__": name})


def _safe_globals():
    """(stand-in, 'module.Name') pairs for torch.serialization.safe_globals plus the plain
    containers an nn.Module pickle holds."""
    pairs = [(_record_type(*_REF_NP), ".".join(_REF_NP)), (_record_type(*_REF_CFG), ".".join(_REF_CFG))]
    pairs += [(_record_type(m, n), f"{m}.{n}") for m, n in _REF_ENCODERS]
    extra = [collections.OrderedDict, set, torch.device]
    np_core = getattr(np, "_core", None) or np.core
    extra += [np_core.multiarray._reconstruct, np.ndarray, np.dtype, type(np.dtype(np.float64)),
              type(np.dtype(np.float32)), type(np.dtype(np.int64)), type(np.dtype(np.bool_)),
              np_core.multiarray.scalar]
    return pairs + extra


def _load_dict(path):
    with torch.serialization.safe_globals(_safe_globals()):
        return torch.load(path, map_location="cpu", weights_only=True)


def _config_from(ref_cfg_state, device):
    """This package's Config with every attribute of the reference's Config copied over
    (the drop-in classes read the same attribute names)."""
    cfg = Config()
    for k, v in ref_cfg_state.items():
        if isinstance(v, _Record):
            continue
        setattr(cfg, k, v)
    cfg.device = device
    return cfg


def load_pin_map(path, device="cuda", config=None):
    """Read a reference ``pin_map.pth`` (or one written by ``save_implicit_map`` here).

    Returns a dict with ``"neural_points"`` (a ``pin_slam_amd.NeuralPoints`` holding the
    map on ``device``), ``"config"`` (the map's configuration: the file's own reference
    Config attributes over this package's defaults, unless ``config`` is given) and the
    decoder state dicts present in the file (``"geo_decoder"``, ``"color_decoder"``,
    ``"sem_decoder"``), loadable into ``pin_slam_amd.Decoder`` unchanged.
    """
    d = _load_dict(path)
    rec = d.get("neural_points")
    if not isinstance(rec, _Record):
        raise ValueError(f"{path}: 'neural_points' is not a pickled model.neural_points.NeuralPoints")
    st = rec.state
    if config is None:
        cstate = st.get("config").state if isinstance(st.get("config"), _Record) else {}
        config = _config_from(cstate, device)
    config.device = device
    # sizes the reference derives from its config at construction
    if "buffer_size" in st:
        config.buffer_size = int(st["buffer_size"])
    if "resolution" in st:
        config.voxel_size_m = float(st["resolution"])
    nm = NeuralPoints(config)
    params = st.get("_parameters") or {}
    install_map_state(nm, st, params, device)
    out = {"neural_points": nm, "config": config}
    for k in ("geo_decoder", "color_decoder", "sem_decoder"):
        if k in d:
            out[k] = {n: t.to(device) for n, t in d[k].items()}
    return out


def install_map_state(nm, st, params, device):
    """Copy the map tensors of a reference NeuralPoints state dict into ``nm`` (device tensors;
    the hash table int64 -> int32, values < buffer_size < 2^31)."""
    def dev(t):
        return t.detach().to(device) if isinstance(t, torch.Tensor) else t

    table = st.get("buffer_pt_index")
    if table is not None:
        if table.numel() != nm.buffer_size:
            raise ValueError(f"hash table has {table.numel()} slots, config.buffer_size is {nm.buffer_size}")
        nm.buffer_pt_index = table.to(device=device, dtype=torch.int32)
    for k in _MAP_TENSORS:
        if k in st:
            setattr(nm, k, dev(st[k]))
    for k in _MAP_SCALARS:
        if k in st:
            setattr(nm, k, st[k])
    nm.buffer_size = int(nm.buffer_size)
    for k in ("local_geo_features", "local_color_features"):
        p = params.get(k) if isinstance(params, dict) else None
        if p is not None:
            setattr(nm, k, torch.nn.Parameter(p.detach().to(device)))
    nm._cache = {}
    # resolution / buffer_size may come from the file: the neighbourhood tables derived from the
    # constructor's values (max_valid_dist2, slot offsets, grid exactness) are rebuilt
    nm._nbhd_cache = {}
    nm._nbhd_key = None
    nm.set_search_neighborhood(num_nei_cells=nm.config.num_nei_cells, search_alpha=nm.config.search_alpha)
    return nm


# ------------------------------------------------------------------ writer
def _module_dict(params, modules):
    """The bookkeeping entries of a pickled torch.nn.Module's __dict__ (nn.Module.__setstate__
    back-fills any hook dict that is missing)."""
    od = collections.OrderedDict
    return {"training": True, "_parameters": od(params), "_buffers": od(), "_non_persistent_buffers_set": set(),
            "_backward_pre_hooks": od(), "_backward_hooks": od(), "_is_full_backward_hook": None,
            "_forward_hooks": od(), "_forward_hooks_with_kwargs": od(), "_forward_hooks_always_called": od(),
            "_forward_pre_hooks": od(), "_forward_pre_hooks_with_kwargs": od(), "_state_dict_hooks": od(),
            "_state_dict_pre_hooks": od(), "_load_state_dict_pre_hooks": od(), "_load_state_dict_post_hooks": od(),
            "_modules": od(modules)}


def _reduce_as_reference(self, protocol):
    import copyreg
    return copyreg.__newobj__, (type(self),), self.__dict__["_pickle_state"]


def _ref_class(module, name):
    """A class that pickles under the reference's path ``module.name`` as ``cls.__new__`` +
    state (how an nn.Module / plain object is pickled)."""
    return type(name, (), {"__module__": module, "__qualname__": name, "__reduce_ex__": _reduce_as_reference})


def _Pickled(cls, state):
    obj = object.__new__(cls)
    obj.__dict__["_pickle_state"] = state
    return obj


def _config_state(config):
    st = {}
    for k, v in vars(config).items():
        if isinstance(v, (bool, int, float, str, type(None), list, tuple, dict, torch.dtype)):
            st[k] = v
    st["device"] = str(getattr(config, "device", "cuda"))
    return st


def save_implicit_map(run_path, neural_points, geo_decoder, color_decoder=None, sem_decoder=None,
                      tensor_device=None):
    """utils/tools.py:224-238: write ``run_path/model/pin_map.pth`` (+ ``memory_footprint.npy``)
    in the reference's format.  ``tensor_device`` moves the saved tensors (e.g. "cpu" for a
    file that loads without a GPU); by default they keep their device, as in the reference."""
    nm = neural_points

    def t(x):
        if not isinstance(x, torch.Tensor):
            return x
        x = x.detach()
        if x.untyped_storage().nbytes() != x.numel() * x.element_size():
            x = x.clone()    # a prefix view of a capacity buffer (NeuralPoints._append_rows): save its rows only
        return x.to(tensor_device) if tensor_device is not None else x

    state = {}
    cfg_cls = _ref_class(*_REF_CFG)
    state.update(_module_dict(
        {"local_geo_features": torch.nn.Parameter(t(nm.local_geo_features)),
         "local_color_features": torch.nn.Parameter(t(nm.local_color_features))}, {}))
    cfg = nm.config
    state["config"] = _Pickled(cfg_cls, _config_state(cfg))
    state.update({
        "silence": bool(getattr(cfg, "silence", True)), "geo_feature_dim": int(nm.geo_feature_dim),
        "geo_feature_std": float(getattr(cfg, "feature_std", 0.0)), "color_feature_dim": int(nm.geo_feature_dim),
        "color_feature_std": float(getattr(cfg, "feature_std", 0.0)), "mean_grid_sampling": False,
        "device": str(tensor_device or getattr(cfg, "device", "cuda")), "dtype": nm.dtype,
        "idx_dtype": torch.int64, "primes": t(nm.primes.to(torch.int64)),
        "buffer_pt_index": t(nm.buffer_pt_index.to(torch.int64)),
        "neighbor_dx": t(nm.neighbor_dx), "neighbor_K": int(nm.neighbor_K),
        "max_valid_dist2": float(nm.max_valid_dist2),
    })
    for k in _MAP_TENSORS:
        if hasattr(nm, k):
            state[k] = t(getattr(nm, k))
    for k in _MAP_SCALARS:
        if hasattr(nm, k):
            state[k] = getattr(nm, k)
    state["memory_footprint"] = list(getattr(nm, "memory_footprint", []))
    map_dict = {"neural_points": _Pickled(_ref_class(*_REF_NP), state), "geo_decoder": geo_decoder.state_dict()}
    if color_decoder is not None:
        map_dict["color_decoder"] = color_decoder.state_dict()
    if sem_decoder is not None:
        map_dict["sem_decoder"] = sem_decoder.state_dict()
    os.makedirs(os.path.join(run_path, "model"), exist_ok=True)
    path = os.path.join(run_path, "model", "pin_map.pth")
    with _reference_modules(cfg_cls, type(map_dict["neural_points"])):
        torch.save(map_dict, path)
    np.save(os.path.join(run_path, "memory_footprint.npy"), np.array(state["memory_footprint"]))
    return path


class _reference_modules:
    """Make the reference's module paths resolvable to the writer's class stubs while pickling
    (pickle checks that a class is importable under its __module__), without replacing a real
    reference module that is already imported."""

    def __init__(self, cfg_cls, np_cls):
        self.entries = [("utils.config", "Config", cfg_cls), ("model.neural_points", "NeuralPoints", np_cls)]
        self.added = []
        self.patched = []

    def __enter__(self):
        for mod, name, cls in self.entries:
            for parent in (mod.split(".")[0], mod):
                if parent not in sys.modules:
                    sys.modules[parent] = types.ModuleType(parent)
                    self.added.append(parent)
            m = sys.modules[mod]
            self.patched.append((m, name, m.__dict__.get(name, _MISSING)))
            setattr(m, name, cls)
        return self

    def __exit__(self, *exc):
        for m, name, old in reversed(self.patched):
            if old is _MISSING:
                delattr(m, name)
            else:
                setattr(m, name, old)
        for mod in reversed(self.added):
            sys.modules.pop(mod, None)
        return False


_MISSING = object()
