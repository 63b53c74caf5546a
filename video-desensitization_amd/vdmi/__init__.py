"""vdmi — MI355X-native detect-and-blur hot path of Video-desensitization.

Host-side mirror of the reference's per-frame interfaces over libvdmi.so
(include/vdmi.h):

* ``Retinaface``                       detect_face/face.py:14-150
* ``YOLO`` / ``PlateDetector``         ultralytics call at combine_detect.py:217,872
* ``mosaic_rectangle_region_single``   combine_detect.py:138-161
* ``batch_process_images``             combine_detect.py:183-277 (hot-loop body on GPU)
* ``Context``                          the C-ABI context (device frames, timing hooks)
"""
from ._lib import VdCapacityError, VdError, load  # noqa: F401
from .context import Context, DeviceBoxes, jpeg_info  # noqa: F401
from .face import Retinaface  # noqa: F401
from .mosaic import mosaic_frames, mosaic_rectangle_region_single  # noqa: F401
from .plate import YOLO, PlateDetector  # noqa: F401

__all__ = ["Context", "DeviceBoxes", "Retinaface", "YOLO", "PlateDetector", "mosaic_rectangle_region_single",
           "mosaic_frames", "VdError", "VdCapacityError", "load", "jpeg_info"]
