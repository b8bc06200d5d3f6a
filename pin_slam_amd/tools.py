"""Drop-ins for the per-point helpers of utils/tools.py on the tracker / mapper input path."""
import torch

from . import _lib
from .mapper import transform_batch_torch  # noqa: F401  (utils/tools.py:401-407)
from .tracker import transform_torch  # noqa: F401  (utils/tools.py:386-399)


def deskewing(points: torch.Tensor, ts: torch.Tensor, pose: torch.Tensor, ts_mid_pose=0.5):
    """utils/tools.py:540-567: motion undistortion of a scan, in place (the reference writes
    through ``points_deskewd = points``).  One launch (pin_deskew); min / max of ts stay on the
    device (torch.aminmax), so nothing syncs."""
    if ts is None:
        return points
    _lib.require_device(points)
    if points.dtype != torch.float32 or not points.is_contiguous():
        raise RuntimeError("deskewing: points must be a contiguous float32 device tensor")
    t = ts.reshape(-1).to(torch.float32).contiguous()
    mm = torch.stack(torch.aminmax(t))
    T = pose.detach().to(device=points.device, dtype=torch.float32).contiguous()
    _lib.call("pin_deskew", _lib.ptr(points), points.shape[0], points.shape[1], _lib.ptr(t), _lib.ptr(mm),
              _lib.ptr(T), float(ts_mid_pose), _lib.stream())
    return points
