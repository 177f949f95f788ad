"""MI355X-native (gfx950) extract -> match -> pose hot path of Bohdanok/ACS_Visual_Odometry.

The compute path is libvo_mi355x.so (HIP kernels + C ABI, include/vo_mi355x.h); this
package is the host-side mirror of the reference interface over that ABI.
"""
from ._lib import LIB_PATH, STATUS, load
from .visual_odometry import Context, DeviceFrames, HostFrames, VisualOdometry, pack_descriptor, unpack_descriptor

__all__ = ["LIB_PATH", "STATUS", "load", "Context", "DeviceFrames", "HostFrames", "VisualOdometry", "pack_descriptor",
           "unpack_descriptor"]
