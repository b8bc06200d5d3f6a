"""pin_slam_amd -- MI355X-native neural-point SDF query / training engine for the
hot path of PIN-SLAM (kelly7707/PIN_SLAM).

Drop-in classes mirror the reference's Python API:
    pin_slam_amd.NeuralPoints   <- model/neural_points.py:NeuralPoints
    pin_slam_amd.Decoder        <- model/decoder.py:Decoder
The compute runs in hand-written HIP kernels for gfx950 (libpin_slam_amd.so,
C ABI in include/pin_slam_amd.h).
"""
from .config import Config
from .decoder import Decoder
from .neural_points import NeuralPoints
from .query import query_sdf

__all__ = ["Config", "Decoder", "NeuralPoints", "query_sdf"]
