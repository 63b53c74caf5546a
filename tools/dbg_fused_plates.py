"""Debug: fused vd_process plate / face boxes vs the drop-in detectors (fp32 s2d plate stem)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-desensitization_amd"))
import numpy as np
import vdmi
from vdmi import synth, weights
from vdmi.pipeline import fused_context

frames = [synth.frame(1080, 1920, i, seed=8) for i in range(3)]
face = vdmi.Retinaface(input_shape=[640, 640, 3], nms_iou=0.4, max_batch=4, weights=weights.retinaface_state_dict(0))
plate = vdmi.YOLO(weights="random", max_batch=4)
ctx = fused_context(face, plate, 2)
fr = np.stack(frames[:2])
raw_fused = ctx.plate_raw(fr)
raw_drop = plate.ctx.plate_raw(fr)
print("plate raw fused vs drop-in max rel", float(np.abs(raw_fused - raw_drop).max() / (np.abs(raw_drop).max() + 1e-9)))
for i, img in enumerate(frames[:2]):
    pb = plate([img])[0].boxes.xyxy.tolist()
    fb = face.detect_images([img])[0][1]
    print(i, "dropin faces", len(fb), "plates", len(pb))
from vdmi import _lib
for fl, nm in ((_lib.VD_PROC_FACES | _lib.VD_PROC_PLATES | _lib.VD_PROC_MOSAIC, "faces+plates"), (_lib.VD_PROC_PLATES, "plates only")):
    out, fa, pl = ctx.process(fr, flags=fl)
    print(nm, "fused plate counts", [int(x) for x in pl.count[:2]], "faces", None if fa is None else [int(x) for x in fa.count[:2]])
    print(nm, "fused plates[0]", pl.frame(0)[0][:3].tolist())
print("dropin plates[0]", plate([frames[0]])[0].boxes.xyxy.tolist()[:3])
