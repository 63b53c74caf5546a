"""Headline benchmark: end-to-end detect+blur FPS on 1920x1080 frames (BASELINE.json).

One step = one batch of B synthetic 1920x1080 RGB frames (already in HBM)
through the whole hot path on each GPU: letterbox -> RetinaFace-R50+FPN+SSH ->
decode/NMS -> box correction -> int() -> mosaic write-back (+ the YOLOv8n
plate forward beside it when --plates). With N GPUs each rank processes its
own B frames (frame sharding, weak scaling) and the per-frame box records are
all-gathered over RCCL. Rank 0 prints one JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 64]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "video-desensitization_amd"))
sys.path.insert(0, ROOT)

PEAK_TFLOPS = {"bf16": 2500.0, "fp16": 2500.0, "fp32": 157.3}   # MI355X_MICROARCH.md: dense MFMA peaks
PEAK_HBM_GBS = 8000.0                           # MI355X_MICROARCH.md: HBM3E spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--plates", type=int, default=-1, help="1: run YOLOv8n beside RetinaFace (default: if built)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip per-kernel HIP event timing")
    ap.add_argument("--faces", type=int, default=1, help="0: plates only, no mosaic (profiling the plate net)")
    return ap.parse_args()


def cpu_baseline(frames, sd, seconds):
    """The CPU oracle (torch-CPU fp32 convs + numpy decode/NMS/mosaic) on a bounded
    sample of the same synthetic frames, on this host's cores."""
    import torch
    from oracle import anchors, bbox, letterbox, mosaic
    from oracle.retinaface import build_oracle_model
    # the GPU box shares its host: use the per-GPU CPU share (OMP_NUM_THREADS, 16 there)
    cores = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    torch.set_num_threads(cores)
    m = build_oracle_model(sd)
    pri = anchors.get_anchors((640, 640))
    done = 0
    t0 = time.perf_counter()
    while done < len(frames):
        img = frames[done]
        x, _ = letterbox.preprocess([img])
        with torch.no_grad():
            loc, cls, _ = m.forward_raw(torch.from_numpy(x))
        _, boxes, _ = bbox.postprocess_frame(loc[0].numpy(), cls[0].numpy(), pri, 0.5, 0.4)
        ib = bbox.truncate_boxes(bbox.correct_and_scale(boxes, img.shape[0], img.shape[1]))
        mosaic.mosaic_frame(img, [tuple(int(v) for v in r) for r in ib], 8)
        done += 1
        if time.perf_counter() - t0 > seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"{done} x {frames.shape[2]}x{frames.shape[1]} synthetic frames through the oracle "
                      f"(torch-CPU fp32 RetinaFace-R50 + numpy decode/NMS/mosaic), {dt:.1f} s"}


def pmc_traffic():
    """HBM bytes per face-conv launch measured by the committed rocprofv3 PMC passes
    of this same command (profiles/rNN_pmc_traffic.json, tools/pmc_traffic.py);
    (None, None) when no such profile exists."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                          "r*_pmc_traffic.json")))
    if not files:
        return None, None, None
    d = json.load(open(files[-1]))
    src = os.path.join("profiles", os.path.basename(files[-1]))
    blur = (d.get("mosaic_out_kernel") or {}).get("traffic_bytes_per_launch")
    return d.get("traffic_bytes_per_launch"), src, blur


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    import vdmi
    from vdmi import synth, weights
    from vdmi import _lib

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")

    B, H, W = a.batch, a.height, a.width
    ctx = vdmi.Context(device=local, precision=a.precision, max_batch=B)
    sd = weights.retinaface_state_dict(0)
    ctx.load_weights(_lib.VD_NET_RETINAFACE, sd)
    plates = a.plates
    if plates != 0:
        try:
            ctx.load_weights(_lib.VD_NET_YOLOV8N, weights.yolov8n_state_dict(0))
            plates = 1
        except vdmi.VdError:
            if plates == 1:
                raise
            plates = 0
    flags = _lib.VD_PROC_FACES | _lib.VD_PROC_MOSAIC | (_lib.VD_PROC_PLATES if plates else 0)
    if not a.faces:
        flags = _lib.VD_PROC_PLATES

    # synthetic frames, distinct per rank, resident in HBM before timing
    host = synth.frames(B, H, W, seed=0, start=rank * B)
    frames = torch.from_numpy(host).to(dev)
    out = torch.empty_like(frames)
    cap = 256
    faces = vdmi.DeviceBoxes(B, cap, dev)
    pboxes = vdmi.DeviceBoxes(B, cap, dev) if plates else None
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    from vdmi.dist import all_gather_records, pack_records
    rec_cap = 64                      # box record: count + 64 boxes per frame

    def step():
        ctx.process(frames, out, faces=faces, plates=pboxes, flags=flags)
        if world > 1:   # per-frame box records -> every rank (RCCL all-gather over xGMI)
            all_gather_records(pack_records(faces.count, faces.xyxy, rec_cap))

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    def timed():
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        d = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([d], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            d = float(t.item())
        return d

    # `value`: the K steps with nothing but the work in the stream (no per-launch
    # events -- recording ~250 events per step costs ~8 % of the step)
    dt = timed()

    roof = blur = None
    extra = {}
    if not a.no_timing:
        # per-kernel-family durations: the same K steps again, each launch bracketed by
        # HIP events on the stream it runs on (runtime.cpp t_begin / t_end)
        ctx.timing(True)
        ctx.timing_reset()
        if world > 1:
            dist.barrier()
        dt_ev = timed()
        extra["instrumented_ms_per_step"] = round(dt_ev / a.steps * 1e3, 3)
        cms, cn, cflop = ctx.timing_read(_lib.FAM_CONV)
        mms, mn, mbytes = ctx.timing_read(_lib.FAM_MOSAIC)
        lms, ln, lbytes = ctx.timing_read(_lib.FAM_LETTERBOX)
        pms, pn, _ = ctx.timing_read(_lib.FAM_POST)
        oms, on_, _ = ctx.timing_read(_lib.FAM_OTHER)
        yms, yn, yflop = ctx.timing_read(_lib.FAM_PLATE_CONV)
        ach = cflop / (cms * 1e-3) / 1e12 if cms > 0 else 0.0
        traffic, tsrc, blur_traffic = pmc_traffic()
        roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": PEAK_TFLOPS[a.precision], "unit": "TFLOP/s",
                "frac": round(ach / PEAK_TFLOPS[a.precision], 4), "traffic": traffic,
                "kernel": "RetinaFace conv family: stem_pool + bottleneck (fused layer1) + chain (layer2) + conv_big + conv_igemm + "
                          "conv1x1_stream launches of a step (the plate net runs concurrently on a second stream)",
                "avg_launch_ms": round(cms / max(cn, 1), 4), "launches": cn,
                "flop_per_launch": round(cflop / max(cn, 1)), "traffic_unit": "bytes per launch (HBM, PMC)",
                "traffic_source": tsrc}
        # blur: the output pass (mosaic_out_kernel) is the dominant kernel; algorithmic bytes
        # per launch = 2*W*H*3 per frame (out-of-place, reference new-array semantics).
        # The family adds the cell-table kernel (box prep + walked cell colours).
        cms6, cn6, _ = ctx.timing_read(_lib.FAM_MOSAIC_CELLS)
        bach = mbytes / (mms * 1e-3) / 1e9 if mms > 0 else 0.0
        fach = mbytes / ((mms + cms6) * 1e-3) / 1e9 if mms > 0 else 0.0
        blur = {"bound": "hbm", "achieved": round(bach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(bach / PEAK_HBM_GBS, 4), "avg_launch_ms": round(mms / max(mn, 1), 4),
                "bytes_per_launch": round(mbytes / max(mn, 1)), "kernel": "mosaic_out_kernel",
                "traffic": blur_traffic, "traffic_source": tsrc,
                "family": {"kernels": "mosaic_cell_kernel + mosaic_out_kernel", "achieved": round(fach, 1),
                           "frac": round(fach / PEAK_HBM_GBS, 4),
                           "avg_ms_per_step": round((mms + cms6) / max(mn, 1), 4)}}
        steps = max(a.steps, 1)
        if yn:
            extra["plate_conv"] = {"achieved_tflops": round(yflop / (yms * 1e-3) / 1e12, 2), "launches": yn,
                                   "avg_launch_ms": round(yms / yn, 4)}
        extra["ms_breakdown_per_step"] = {"conv": round(cms / steps, 3), "plate_conv": round(yms / steps, 3),
                                          "mosaic": round((mms + cms6) / steps, 3),
                                          "letterbox": round(lms / steps, 3), "post": round(pms / steps, 3),
                                          "other": round(oms / steps, 3)}
        ctx.timing(False)

    total_frames = world * B * a.steps
    value = total_frames / dt
    res = {
        "metric": "end-to-end detect+blur FPS on 1920x1080 frames",
        "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": a.precision, "data": "synthetic (counter-hash frames, seeded random weights)",
        "config": {"workload": f"RetinaFace-R50+FPN+SSH{' + YOLOv8n plates' if plates else ''} detect + mosaic "
                               f"write-back, batch={B} frames of {W}x{H} per GPU",
                   "global_batch": world * B, "frame": f"{W}x{H}", "net_input": "640x640",
                   "parallelism": f"frame-sharded x{world}" + (", RCCL all-gather of box records" if world > 1 else ""),
                   "plates": bool(plates)},
        "roofline": roof, "blur_roofline": blur,
        "faces_per_frame": round(float(faces.count.float().mean().item()), 2),
    }
    res.update(extra)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(host[:64], sd, a.cpu_baseline_seconds)
    if rank == 0:
        print(json.dumps(res), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
