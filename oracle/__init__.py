"""CPU oracle for the detect-and-blur hot path — TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU, what the reference computes on the path
``letterbox -> RetinaFace-R50 forward -> decode + NMS -> box correction ->
int() truncation -> sequential mosaic`` (plus the YOLOv8n plate forward that
runs beside it). It is the checker, never the product:

* only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
  ``cpu_baseline`` leg may import it;
* nothing under ``video-desensitization_amd/`` imports it, and the product
  path fails loudly when its HIP library is missing.

Provenance of each rule (every function cites the reference file:line it
follows, paths relative to the reference repository root):

* anchors          detect_face/utils/anchors.py:22-41, utils/config.py:18-29
* letterbox        detect_face/utils/utils.py:8-18,27-28, detect_face/face.py:65-88
                   (+ OpenCV 4.9.0.80 ``cv2.resize`` INTER_LINEAR / area-fast, [ext])
* network          detect_face/retinaface.py:13-148, detect_face/nets/layers.py:10-114
                   (+ torchvision 0.22.1 ``resnet50`` topology, [ext])
* decode / NMS     detect_face/utils/utils_bbox.py:49-79,103-130, face.py:93-115
                   (+ torchvision ``batched_nms`` CPU kernel semantics, [ext])
* correction       detect_face/utils/utils_bbox.py:12-43, face.py:136-150,
                   combine_detect.py:243
* mosaic           combine_detect.py:138-161,247-249 (+ OpenCV ``resizeNN``, [ext])
* plate detector   combine_detect.py:9,217,872 (ultralytics YOLOv8n, [ext], version
                   unpinned by the reference)

Pinning: the reference ships no tests, fixtures or golden vectors (SURVEY.md
§4, §8c) and importing/running it in this environment was refused (SURVEY.md
§8c; binding on every later round). The oracle is therefore pinned by
hand-derived known-answer tests written from the reference source text
(``tests/test_oracle_kat.py``) and by golden fixtures it generates itself
(``tests/golden/``, script ``tools/make_golden.py``). Third-party arithmetic
(OpenCV resize rounding outside the integer-ratio cases, torchvision NMS tie
order on the >4000-element path, ultralytics post-processing) is restated from
upstream behaviour and is **parity unpinned** by the reference itself.
"""
