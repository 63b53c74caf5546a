"""batch_process_images mirror (combine_detect.py:183-277) end to end on the GPU,
with in-memory loader/saver (cv2 is absent), against the oracle's per-box mosaic
of the detector outputs; plus the drop-the-batch error path (:226-228)."""
import os

import numpy as np
import pytest

from oracle import mosaic as omosaic

pytestmark = pytest.mark.gpu


def test_batch_process_images(gpu, tmp_path):
    import vdmi
    from vdmi import synth, weights
    from vdmi.pipeline import batch_process_images
    frames = {f"f{i:03d}.jpg": synth.frame(360, 640, i, seed=3) for i in range(7)}
    for name in frames:
        (tmp_path / name).write_bytes(b"")          # the listing drives the batch order
    saved = {}
    face = vdmi.Retinaface(input_shape=[640, 640, 3], nms_iou=0.4, max_batch=4, weights=weights.retinaface_state_dict(0))
    plate = vdmi.YOLO(weights="random", max_batch=4)
    n, nf, npl = batch_process_images(str(tmp_path), str(tmp_path / "out"), face, plate, batch_size=3,
                                      loader=lambda p: frames[os.path.basename(p)],
                                      saver=lambda img, p: saved.__setitem__(os.path.basename(p), img))
    assert n == 7 and npl == 0             # plate Results are not tuples: discarded like the reference
    assert len(saved) == 7
    total = 0
    for name, img in frames.items():
        boxes = face.detect_images([img])[0][1]
        total += len(boxes)
        exp = omosaic.mosaic_frame(img, [tuple(int(v) for v in b) for b in boxes], 8)
        np.testing.assert_array_equal(saved[f"processed_{name}"], exp)
    assert nf == total


def test_batch_dropped_on_inference_error(gpu, tmp_path):
    import vdmi
    from vdmi import synth, weights
    from vdmi.pipeline import batch_process_images

    class Boom:
        def __call__(self, *a, **k):
            raise RuntimeError("plate model failure")

    (tmp_path / "a.png").write_bytes(b"")
    face = vdmi.Retinaface(input_shape=[640, 640, 3], max_batch=2, weights=weights.retinaface_state_dict(0))
    saved = {}
    n, nf, npl = batch_process_images(str(tmp_path), str(tmp_path / "o"), face, Boom(), batch_size=4,
                                      loader=lambda p: synth.frame(64, 64, 0),
                                      saver=lambda img, p: saved.__setitem__(p, img))
    assert (n, nf, npl) == (0, 0, 0) and not saved
