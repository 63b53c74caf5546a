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


def test_frame_pipeline_matches_unpipelined_process(gpu):
    """FramePipeline (pinned double buffers, upload / compute / download streams,
    results one batch behind) == one synchronous vd_process per batch: same
    mosaicked pixels, complete counts and boxes, for faces and plates, incl. a
    short last batch."""
    import vdmi
    from vdmi import _lib, synth, weights
    from vdmi.pipeline import FramePipeline
    ctx = vdmi.Context(precision="bf16", max_batch=4)
    try:
        ctx.load_weights(0, weights.retinaface_state_dict(0))
        ctx.load_weights(1, weights.yolov8n_state_dict(0))
        batches = [synth.frames(4, 1080, 1920, seed=40, start=4 * i) for i in range(3)] + \
                  [synth.frames(2, 1080, 1920, seed=41)]
        pipe = FramePipeline(ctx, 1080, 1920, max_batch=4, mosaic_plates=True)
        got = [(o.copy(), fc.copy(), [b.copy() for b in fb], pc.copy(), [b.copy() for b in pb])
               for o, fc, fb, pc, pb in pipe.run(iter(batches))]
        pipe.close()
        flags = _lib.VD_PROC_FACES | _lib.VD_PROC_PLATES | _lib.VD_PROC_MOSAIC | _lib.VD_PROC_MOSAIC_PLATES
        assert len(got) == len(batches)
        nf = 0
        for fr, (o, fc, fb, pc, pb) in zip(batches, got):
            out, faces, plates = ctx.process(fr, flags=flags)
            np.testing.assert_array_equal(o, out)
            np.testing.assert_array_equal(fc, faces.count)
            np.testing.assert_array_equal(pc, plates.count)
            for j in range(fr.shape[0]):
                np.testing.assert_array_equal(fb[j], faces.frame(j)[0])
                np.testing.assert_array_equal(pb[j], plates.frame(j)[0])
            nf += int(fc.sum())
        assert nf > 0
    finally:
        ctx.close()


def test_batch_process_images_fused_mosaic_plates(gpu, tmp_path):
    """The fused path with mosaic_plates=True (intended mode): plates are counted and
    blurred after the faces, exactly as the oracle's sequential mosaic of the drop-in
    detectors' boxes (faces in NMS order, then plates)."""
    import vdmi
    from vdmi import synth, weights
    from vdmi.pipeline import batch_process_images
    frames = {f"g{i:02d}.png": synth.frame(1080, 1920, i, seed=8) for i in range(3)}
    for name in frames:
        (tmp_path / name).write_bytes(b"")
    saved = {}
    face = vdmi.Retinaface(input_shape=[640, 640, 3], nms_iou=0.4, max_batch=4,
                           weights=weights.retinaface_state_dict(0))
    plate = vdmi.YOLO(weights="random", max_batch=4)
    n, nf, npl = batch_process_images(str(tmp_path), str(tmp_path / "out"), face, plate, batch_size=2,
                                      loader=lambda p: frames[os.path.basename(p)], mosaic_plates=True,
                                      saver=lambda img, p: saved.__setitem__(os.path.basename(p), img))
    assert n == 3 and len(saved) == 3
    tf = tp = 0
    for name, img in frames.items():
        fb = face.detect_images([img])[0][1]
        pb = plate([img])[0].boxes.xyxy.tolist()
        tf += len(fb)
        tp += len(pb)
        boxes = [tuple(int(v) for v in b) for b in fb] + [tuple(int(v) for v in b) for b in pb]
        np.testing.assert_array_equal(saved[f"processed_{name}"], omosaic.mosaic_frame(img, boxes, 8))
    assert (nf, npl) == (tf, tp) and tp > 0


def test_batch_process_images_gpu_jpeg_codec(gpu, tmp_path):
    """The reference's real file loop: a directory of ffmpeg-style JPEG frames (q95
    4:2:0) -> batch_process_images with vdmi detectors and no custom I/O takes the GPU
    codec path (vd_jpeg_decode -> vd_process -> vd_jpeg_encode). Every written file is
    byte-identical to libjpeg-turbo's encode (Pillow, q95, 4:2:0) of the oracle mosaic
    of the host-decoded frame with the detector's boxes; a progressive JPEG among them
    takes the host decoder and is still processed."""
    import io
    from PIL import Image
    import vdmi
    from vdmi import synth, weights
    from vdmi.pipeline import batch_process_images
    src = {}
    for i in range(7):
        img = np.repeat(np.repeat(synth.frame(180, 320, i, seed=5), 2, 0), 2, 1)   # 360x640, real structure
        b = io.BytesIO()
        Image.fromarray(img).save(b, "JPEG", quality=95, progressive=(i == 6))
        (tmp_path / f"f{i:03d}.jpg").write_bytes(b.getvalue())
        src[f"f{i:03d}.jpg"] = np.asarray(Image.open(io.BytesIO(b.getvalue())).convert("RGB"))
    face = vdmi.Retinaface(input_shape=[640, 640, 3], nms_iou=0.4, max_batch=4,
                           weights=weights.retinaface_state_dict(0))
    plate = vdmi.YOLO(weights="random", max_batch=4)
    out_dir = tmp_path / "out"
    n, nf, npl = batch_process_images(str(tmp_path), str(out_dir), face, plate, batch_size=3)
    assert n == 7 and npl == 0
    total = 0
    for name, img in src.items():
        boxes = face.detect_images([img])[0][1]
        total += len(boxes)
        exp = omosaic.mosaic_frame(img, [tuple(int(v) for v in b) for b in boxes], 8)
        b = io.BytesIO()
        Image.fromarray(exp).save(b, "JPEG", quality=95, subsampling=2)
        assert (out_dir / f"processed_{name}").read_bytes() == b.getvalue(), name
    assert nf == total and total > 0


def test_batch_process_images_two_frame_sizes(gpu, tmp_path):
    """Frames of two sizes in one folder: the fused path opens one FramePipeline per
    size on ONE shared context, each submission re-binds the context to its own
    compute stream (the one that waited on that slot's upload). Every saved frame
    equals the oracle mosaic of the drop-in detector's boxes (none is left
    unmosaicked by a stream race)."""
    import vdmi
    from vdmi import synth, weights
    from vdmi.pipeline import batch_process_images
    frames = {}
    for i in range(8):
        h, w = (720, 1280) if i % 2 else (1080, 1920)
        frames[f"m{i:02d}.png"] = np.repeat(np.repeat(synth.frame(h // 2, w // 2, i, seed=12), 2, 0), 2, 1)
    for name in frames:
        (tmp_path / name).write_bytes(b"")
    saved = {}
    face = vdmi.Retinaface(input_shape=[640, 640, 3], nms_iou=0.4, max_batch=4,
                           weights=weights.retinaface_state_dict(0))
    plate = vdmi.YOLO(weights="random", max_batch=4)
    n, nf, _ = batch_process_images(str(tmp_path), str(tmp_path / "out"), face, plate, batch_size=4,
                                    loader=lambda p: frames[os.path.basename(p)],
                                    saver=lambda img, p: saved.__setitem__(os.path.basename(p), img))
    assert n == 8 and len(saved) == 8
    total = 0
    for name, img in frames.items():
        boxes = face.detect_images([img])[0][1]
        total += len(boxes)
        exp = omosaic.mosaic_frame(img, [tuple(int(v) for v in b) for b in boxes], 8)
        np.testing.assert_array_equal(saved[f"processed_{name}"], exp, err_msg=name)
    assert nf == total and total > 0


def test_batch_process_images_load_failure_aborts(gpu, tmp_path):
    """combine_detect.py:209-211: the loader runs outside the inference try, so an
    unreadable frame aborts the call; the batches submitted before it are still
    finished and saved."""
    import vdmi
    from vdmi import synth, weights
    from vdmi.pipeline import batch_process_images
    for i in range(6):
        (tmp_path / f"x{i}.png").write_bytes(b"")
    saved = {}

    def loader(p):
        if os.path.basename(p) == "x5.png":
            raise ValueError(f"cannot read image: {p}")
        return synth.frame(360, 640, 1, seed=2)

    face = vdmi.Retinaface(input_shape=[640, 640, 3], max_batch=1, weights=weights.retinaface_state_dict(0))
    plate = vdmi.YOLO(weights="random", max_batch=1)
    with pytest.raises(ValueError, match="cannot read"):
        batch_process_images(str(tmp_path), str(tmp_path / "o"), face, plate, batch_size=1, loader=loader,
                             saver=lambda img, p: saved.__setitem__(os.path.basename(p), img))
    listed = [f for f in os.listdir(tmp_path) if f.endswith(".png")]
    assert len(saved) == listed.index("x5.png")      # every batch listed before the bad frame


def test_gpu_jpeg_stages_serial_decode_equals_overlapped(gpu):
    """GpuJpegStages with decode(i + 1) held back until process(i) has finished
    (decode_overlap=False; "auto" picks it after a decode with many resynchronisation
    passes) writes the same JPEG bytes, face counts and job order as the overlapped
    schedule."""
    import vdmi
    from vdmi import _lib, synth, weights
    from vdmi.pipeline import GpuJpegStages
    ctx = vdmi.Context(device=0, precision="fp32", max_batch=4)
    ctx.load_weights(_lib.VD_NET_RETINAFACE, weights.retinaface_state_dict(0))
    frames = [np.stack([np.repeat(np.repeat(synth.frame(180, 320, 4 * j + k, seed=5), 2, 0), 2, 1) for k in range(4)])
              for j in range(4)]
    frames[1] = synth.frames(4, 360, 640, seed=9)                      # noise: many passes
    import torch
    blobs = [[bytes(b) for b in ctx.jpeg_encode(torch.from_numpy(f).cuda(), quality=95, subsampling=2)]
             for f in frames]
    flags = _lib.VD_PROC_FACES | _lib.VD_PROC_MOSAIC
    got = {}
    for mode in (True, False, "auto"):
        st = GpuJpegStages(ctx, 4, flags, quality=95, subsampling=2, decode_overlap=mode)
        out = []
        try:
            st.run(((j, (lambda j=j: blobs[j]), None) for j in range(len(blobs))),
                   lambda key, res, nf, npl: out.append((key, nf, [bytes(b) for _, jp in res for b in jp])))
        finally:
            st.close()
        if mode is False:
            assert st.serial_jobs == len(blobs) - 1
        got[mode] = out
    ctx.close()
    assert [k for k, _, _ in got[True]] == list(range(len(blobs)))
    assert got[False] == got[True] and got["auto"] == got[True]


def test_gpu_jpeg_stages_mixed_sizes_counts(gpu):
    """A job whose frames have two sizes: each size group is processed into its own
    rows of the slot's box lists, so the job's face / plate totals equal the sum of
    per-frame vd_process counts (a shared row range would count the last group twice
    and drop the first), and every frame's JPEG bytes equal the encode of its own
    processed frame."""
    import torch
    import vdmi
    from vdmi import _lib, synth, weights
    from vdmi.pipeline import GpuJpegStages
    ctx = vdmi.Context(device=0, precision="fp32", max_batch=4)
    ctx.load_weights(_lib.VD_NET_RETINAFACE, weights.retinaface_state_dict(0))
    ctx.load_weights(_lib.VD_NET_YOLOV8N, weights.yolov8n_state_dict(0))
    flags = _lib.VD_PROC_FACES | _lib.VD_PROC_PLATES | _lib.VD_PROC_MOSAIC | _lib.VD_PROC_MOSAIC_PLATES
    jobs = []
    for j in range(3):
        fr = []
        for k in range(4):
            h, w = ((360, 640), (720, 1280))[(j + k) % 2 if k < 3 else 1]
            fr.append(np.repeat(np.repeat(synth.frame(h // 2, w // 2, 4 * j + k, seed=21), 2, 0), 2, 1))
        jobs.append(fr)
    blobs = [[bytes(ctx.jpeg_encode(torch.from_numpy(f[None]).cuda(), quality=95, subsampling=2)[0]) for f in fr]
             for fr in jobs]
    got = []
    st = GpuJpegStages(ctx, 4, flags, quality=95, subsampling=2)
    try:
        st.run(((j, (lambda j=j: blobs[j]), None) for j in range(len(blobs))),
               lambda key, res, nf, npl: got.append((key, nf, npl, {k: bytes(b) for idx, jp in res
                                                                     for k, b in zip(idx, jp)})))
    finally:
        st.close()
    assert [g[0] for g in got] == list(range(len(blobs)))
    tf = tp = 0
    for (j, nf, npl, jpegs), fr in zip(got, jobs):
        ef = ep = 0
        for k, b in enumerate(blobs[j]):
            dec = torch.from_numpy(ctx.jpeg_decode([b])).cuda()
            out, faces, plates = ctx.process(dec, flags=flags)
            ef += int(faces.count.sum())
            ep += int(plates.count.sum())
            assert jpegs[k] == bytes(ctx.jpeg_encode(out, quality=95, subsampling=2)[0]), (j, k)
        assert (nf, npl) == (ef, ep), j
        tf += ef
        tp += ep
    ctx.close()
    assert tf > 0
