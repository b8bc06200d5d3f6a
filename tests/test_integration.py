"""pin_slam_amd.integration.install() against stand-in reference modules (CPU): the class
swap and the method transplant land where pin_slam.py / utils/*.py look them up."""
import sys
import types

import pin_slam_amd as P
from pin_slam_amd import integration


def _fake(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    return m


def test_install_patches_reference_modules(monkeypatch):
    class RefMapper:
        def process_frame(self):
            return "reference"

        def bundle_adjustment(self):
            return "kept"

        def mapping(self, n):
            return "reference"

    class RefTracker:
        def tracking(self):
            return "reference"

    class RefMesher:
        def query_points(self):
            return "reference"

        def mc_mesh(self):
            return "reference"

    mods = {"model": _fake("model"), "model.neural_points": _fake("model.neural_points", NeuralPoints=object),
            "model.decoder": _fake("model.decoder", Decoder=object), "utils": _fake("utils"),
            "utils.mapper": _fake("utils.mapper", Mapper=RefMapper, DataSampler=object),
            "utils.data_sampler": _fake("utils.data_sampler", DataSampler=object),
            "utils.tools": _fake("utils.tools", deskewing=object),
            "utils.tracker": _fake("utils.tracker", Tracker=RefTracker),
            "utils.mesher": _fake("utils.mesher", Mesher=RefMesher)}
    for k, v in mods.items():
        monkeypatch.setitem(sys.modules, k, v)
    patched = integration.install()
    from model.neural_points import NeuralPoints
    from model.decoder import Decoder
    assert NeuralPoints is P.NeuralPoints and Decoder is P.Decoder
    assert RefMapper.mapping is P.Mapper.mapping and RefMapper.train_step is P.Mapper.train_step
    assert RefMapper.process_frame is P.Mapper.process_frame and RefMapper().bundle_adjustment() == "kept"
    from pin_slam_amd.data_sampler import DataSampler
    from pin_slam_amd.tools import deskewing
    assert sys.modules["utils.data_sampler"].DataSampler is DataSampler
    assert sys.modules["utils.mapper"].DataSampler is DataSampler
    assert sys.modules["utils.tools"].deskewing is deskewing
    assert RefTracker.tracking is P.Tracker.tracking and RefTracker.registration_step is P.Tracker.registration_step
    assert RefMesher.query_points is P.Mesher.query_points and RefMesher.mc_mesh is P.Mesher.mc_mesh
    assert ("utils.mapper", "Mapper.mapping") in patched
