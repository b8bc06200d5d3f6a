"""Route an unmodified PIN-SLAM checkout's hot path through pin_slam_amd.

    import pin_slam_amd.integration
    pin_slam_amd.integration.install()      # first lines of pin_slam.py / pin_slam_ros.py / vis_pin_map.py

``install()`` imports the reference modules (so it must run where they import) and

* replaces ``model.neural_points.NeuralPoints`` and ``model.decoder.Decoder`` by the drop-in
  classes, so every later ``from model.neural_points import NeuralPoints`` binds ours;
* replaces ``utils.data_sampler.DataSampler`` (and the name ``utils.mapper`` imported) by the
  fused sampler, and ``deskewing`` in ``utils.tools`` / ``dataset.slam_dataset`` by the kernel;
* transplants the hot-path methods onto the reference's ``utils.mapper.Mapper``,
  ``utils.tracker.Tracker`` and ``utils.mesher.Mesher`` classes, together with every helper
  method they call, keeping everything else of those classes as it is.  The reference's own
  control flow (``Mapper.get_batch`` / ``sdf`` /
  ``get_numerical_gradient``, bundle adjustment, ...) stays: it calls the transplanted
  hot-path methods and the drop-in ``NeuralPoints`` / ``Decoder``.

``tests/test_integration.py`` imports the real reference modules, runs ``install()``, builds the
reference ``Mapper`` / ``Tracker`` / ``Mesher`` and checks that every ``self.<name>`` a
transplanted method reads resolves on those instances.

It returns the list of (module, attribute) pairs it patched.  Nothing in the package calls it.
"""
import importlib

from .data_sampler import DataSampler
from .decoder import Decoder
from .mapper import Mapper
from .mesher import Mesher
from .neural_points import NeuralPoints
from .tools import deskewing
from .tracker import Tracker

# utils/mapper.py:Mapper -- the fused training loop (mapping :425-593), the device-resident data
# pool (process_frame :110-321, dynamic_filter :79-108) and the helpers those call
MAPPER_METHODS = ("mapping", "train_step", "_step_index", "_step_plan", "_dense_loop", "_owner_adam", "check_deferred", "_device_seed", "_adam",
                  "_adam_segments", "_check_supported", "_world", "_pools_fusable", "_slab_partition", "_batch_index",
                  "_batch_parts", "_batch_sizes", "_randint", "_new_sample_mode", "process_frame", "dynamic_filter", "_used_poses", "_poses_dev",
                  "_pool_append", "_pool_compact", "_pool_compact_many", "_pool_compact_target", "_window_buffers", "_pool_rows_hint", "set_pool", "_pool_signature", "_pack",
                  "_packed_pool")
# utils/tracker.py:Tracker -- the fused query, the registration step and the tracking loop
# (:39-174) with the pose kept on the device and each iteration enqueued one ahead of the host's
# read of the previous one (tracker._RegLoop), instead of the reference's per-iteration host syncs
TRACKER_METHODS = ("tracking", "_iteration_done", "query_source_points", "registration_step", "_register",
                   "_shard_range")
# utils/mesher.py:Mesher -- grid queries (:41-136) and marching cubes (:310-337)
MESHER_METHODS = ("query_points", "mc_mesh")


def install(neural_points=True, decoder=True, mapper=True, tracker=True, mesher=True, sampler=True):
    patched = []

    def setcls(modname, name, obj, optional=False):
        try:
            mod = importlib.import_module(modname)
        except ImportError:
            if optional:
                return
            raise
        setattr(mod, name, obj)
        patched.append((modname, name))

    def methods(modname, clsname, src, names):
        cls = getattr(importlib.import_module(modname), clsname)
        for n in names:
            setattr(cls, n, src.__dict__[n])
            patched.append((modname, f"{clsname}.{n}"))

    if neural_points:
        setcls("model.neural_points", "NeuralPoints", NeuralPoints)
    if decoder:
        setcls("model.decoder", "Decoder", Decoder)
    if sampler:
        setcls("utils.data_sampler", "DataSampler", DataSampler)
        setcls("utils.mapper", "DataSampler", DataSampler)
        setcls("utils.tools", "deskewing", deskewing)
        setcls("dataset.slam_dataset", "deskewing", deskewing, optional=True)
    if mapper:
        methods("utils.mapper", "Mapper", Mapper, MAPPER_METHODS)
    if tracker:
        methods("utils.tracker", "Tracker", Tracker, TRACKER_METHODS)
    if mesher:
        methods("utils.mesher", "Mesher", Mesher, MESHER_METHODS)
    return patched
