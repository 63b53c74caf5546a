"""Hot-loop body of the reference driver on the MI355X path.

``batch_process_images`` mirrors combine_detect.py:183-277 (same signature, same
per-batch semantics): list the frame files, load a batch, run the face detector
and the plate detector, take face boxes from ``face_results[j][1]`` and plate
boxes from ``plate_results[j][1] if isinstance(..., tuple) else []``
(combine_detect.py:237-239 — Results objects yield [], so plates are discarded
exactly as in the reference unless ``mosaic_plates=True``), truncate with int()
(:243-244), mosaic sequentially per box (:246-249), save, count faces/plates, and
drop a batch whose inference raises (:226-228).

``process_batch`` is the same body on device-resident frames through one
``vd_process`` call (letterbox, both forwards, NMS, mosaic), which is what the
benchmark times. Image I/O (cv2.imread/imwrite, combine_detect.py:167-180) is
outside the hot path; it is used when cv2 is importable and can be replaced by
``loader`` / ``saver`` callables.
"""
import logging
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import _lib
from .mosaic import mosaic_frames

IMAGE_EXT = (".png", ".jpg", ".jpeg")


def _cv2():
    try:
        import cv2
        return cv2
    except Exception as e:  # pragma: no cover - cv2 is absent in this image
        raise RuntimeError("cv2 is needed for file I/O; pass loader=/saver= callables instead") from e


def load_image_rgb(path):
    """combine_detect.py:167-172."""
    cv2 = _cv2()
    img = cv2.imread(path)
    if img is None:
        raise ValueError(f"cannot read image: {path}")
    return cv2.cvtColor(img, cv2.COLOR_BGR2RGB)


def save_output_image(image_array, output_path):
    """combine_detect.py:177-180."""
    cv2 = _cv2()
    cv2.imwrite(output_path, cv2.cvtColor(image_array, cv2.COLOR_RGB2BGR))


def _boxes_of(result):
    return result[1] if isinstance(result, tuple) else []


def batch_process_images(input_dir, output_dir, face_detector, plate_detector, batch_size=16,
                         loader=None, saver=None, mosaic_plates=False, mosaic_level=8, num_workers=6):
    """combine_detect.py:183-277. Returns (total_processed, total_faces, total_plates)."""
    logger = logging.getLogger("VideoProcessor.batch_process_images")
    loader = loader or load_image_rgb
    saver = saver or save_output_image
    image_paths = [os.path.join(input_dir, f) for f in os.listdir(input_dir) if f.lower().endswith(IMAGE_EXT)]
    os.makedirs(output_dir, exist_ok=True)
    total_processed = total_faces = total_plates = 0
    executor = ThreadPoolExecutor(max_workers=num_workers)
    save_futures = []
    for i in range(0, len(image_paths), batch_size):
        batch_files = image_paths[i:i + batch_size]
        with ThreadPoolExecutor(max_workers=num_workers) as pool:
            batch_images = list(pool.map(loader, batch_files))
        with ThreadPoolExecutor(max_workers=2) as infer:   # face || plate, as the reference does
            ff = infer.submit(face_detector.detect_images, batch_images.copy())
            fp = infer.submit(plate_detector, batch_images.copy(), verbose=False, conf=0.5)
            try:
                face_results = ff.result()
                plate_results = fp.result()
            except Exception as e:   # combine_detect.py:226-228: the batch is dropped
                logger.error(f"parallel inference failed: {e}")
                continue
        per_frame = []
        for j in range(len(batch_images)):
            face_boxes = _boxes_of(face_results[j])
            if mosaic_plates and not isinstance(plate_results[j], tuple):
                plate_boxes = plate_results[j].boxes.xyxy.tolist()
            else:
                plate_boxes = _boxes_of(plate_results[j])
            boxes = [(int(x1), int(y1), int(x2), int(y2)) for x1, y1, x2, y2 in face_boxes]
            boxes += [(int(x1), int(y1), int(x2), int(y2)) for x1, y1, x2, y2 in plate_boxes]
            per_frame.append(boxes)
            total_faces += len(face_boxes)
            total_plates += len(plate_boxes)
        processed = _mosaic_grouped(batch_images, per_frame, mosaic_level)
        for path, img in zip(batch_files, processed):
            out = os.path.join(output_dir, f"processed_{os.path.basename(path)}")
            save_futures.append(executor.submit(saver, img, out))
        total_processed += len(batch_files)
    for f in save_futures:
        try:
            f.result()
        except Exception as e:
            logger.error(f"saving failed: {e}")
    executor.shutdown()
    logger.info(f"processed {total_processed} images: {total_faces} faces, {total_plates} plates")
    return total_processed, total_faces, total_plates


def _mosaic_grouped(images, boxes, level):
    """One mosaic launch per same-size group of frames."""
    out = [None] * len(images)
    groups = {}
    for i, im in enumerate(images):
        groups.setdefault(im.shape, []).append(i)
    for idx in groups.values():
        res = mosaic_frames(np.stack([images[i] for i in idx]), [boxes[i] for i in idx], level)
        for k, i in enumerate(idx):
            out[i] = res[k]
    return out


def process_batch(ctx, frames, out=None, faces=None, plates=None, plates_enabled=True, mosaic_plates=False):
    """Device-resident hot path: one vd_process call over a frame batch
    (torch uint8 [n,h,w,3] on the context's GPU, or numpy). Returns (out, faces, plates)."""
    flags = _lib.VD_PROC_FACES | _lib.VD_PROC_MOSAIC
    if plates_enabled:
        flags |= _lib.VD_PROC_PLATES
        if mosaic_plates:
            flags |= _lib.VD_PROC_MOSAIC_PLATES
    return ctx.process(frames, out=out, faces=faces, plates=plates, flags=flags)
