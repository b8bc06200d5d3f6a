"""pin_slam_amd -- MI355X-native neural-point SDF query / training engine for the
hot path of PIN-SLAM (kelly7707/PIN_SLAM).

Drop-in classes mirror the reference's Python API:
    pin_slam_amd.NeuralPoints   <- model/neural_points.py:NeuralPoints
    pin_slam_amd.Decoder        <- model/decoder.py:Decoder
    pin_slam_amd.Mapper         <- utils/mapper.py:Mapper (training path)
    pin_slam_amd.Tracker        <- utils/tracker.py:Tracker (registration path)
    pin_slam_amd.Mesher         <- utils/mesher.py:Mesher.query_points
    pin_slam_amd.load_pin_map / save_implicit_map <- model/pin_map.pth (utils/tools.py:224-238)
The compute runs in hand-written HIP kernels for gfx950 (libpin_slam_amd.so,
C ABI in include/pin_slam_amd.h).
"""
from .config import Config
from .decoder import Decoder
from .mapper import Mapper
from .mesher import Mesher
from .neural_points import NeuralPoints
from .query import query_sdf
from .tracker import Tracker
from .mapio import load_pin_map, save_implicit_map

__all__ = ["Config", "Decoder", "Mapper", "Mesher", "NeuralPoints", "Tracker", "query_sdf", "load_pin_map",
           "save_implicit_map"]
