"""Headline benchmark: end-to-end detect+blur FPS on 1920x1080 frames (BASELINE.json).

One step = one batch of B synthetic 1920x1080 RGB frames (already in HBM)
through the whole hot path on each GPU: letterbox -> RetinaFace-R50+FPN+SSH ->
decode/NMS -> box correction -> int() -> mosaic write-back, with the YOLOv8n
plate forward + NMS beside it (BASELINE config 3).

The headline runs in fp32 -- the reference's arithmetic: f32 activations and
weights. Every conv scales its f32 operands by powers of two (per frame from the
producer's running max |x|, per output channel for the weights) and splits them
into fp16 pairs: three products on the f16 matrix cores, f32 accumulation
(conv_x6.hip), error at f32 level; this is the mode whose boxes are parity-checked
against the oracle. The same frames are then run on the exact 3-term bf16 split
(`fp32_x6`, 6 products), exact-f32 MFMA (`fp32_exact`), bf16 and fp16 (`modes`),
and `parity` reports, over the B bench frames, the fraction whose complete keep
lists and int boxes equal the headline's (and, from the cpu_baseline leg, each fp32
path's agreement with the oracle).

Multi-GPU (one process per GPU, torchrun): `--scaling weak` (default) gives every
rank its own B frames; `--scaling strong --frames N` shards ONE list of N frames
with vdmi.dist.shard_range. Either way the per-frame box records (frame index,
count, boxes, scores, anchors) are all-gathered over RCCL; pixels stay local.
Rank 0 prints one JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 64] [--precision fp32]
    torchrun --nproc-per-node N bench.py --gpus N ...

`python bench.py --gpus N` (N > 1) with no WORLD_SIZE in the environment starts the
N ranks itself: the parent makes no GPU call, runs torch.distributed.run as a child
process (127.0.0.1 rendezvous, a free port) with the same arguments and exits with
its status. A rank errors out when WORLD_SIZE != --gpus. `--force-dist` takes the
distributed path (process group, record all-gather) even at one rank, so the RCCL
branch can be exercised on a one-GPU box.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "video-desensitization_amd"))
sys.path.insert(0, ROOT)

# MI355X_MICROARCH.md dense MFMA peaks. fp32 (default plan, conv_x6.hip): f32 FLOPs on the f16
# matrix cores at three products per multiply-add (scaled fp16 pairs) -> 2500 / 3; fp32_x6 (exact
# 3-term bf16 split, six products) -> 2500 / 6; fp32_exact: v_mfma_f32_16x16x4_f32.
PEAK_TFLOPS = {"bf16": 2500.0, "fp16": 2500.0, "fp32": 2500.0 / 3, "fp32_x6": 2500.0 / 6, "fp32_exact": 157.3}
PEAK_HBM_GBS = 8000.0                           # MI355X_MICROARCH.md: HBM3E spec


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--frames-src", default="noise", choices=["noise", "up2"],
                    help="noise: counter-hash frames at full size; up2: hash frames at half size, 2x nearest "
                         "upsampled (the ratio-2 / ratio-6 letterboxes of 720p / 4K then see structure and the "
                         "seeded weights detect faces; raw noise at those ratios averages out to none)")
    ap.add_argument("--precision", default="fp32", choices=["bf16", "fp16", "fp32", "fp32_x6", "fp32_exact"])
    ap.add_argument("--compare", default="fp32_x6,fp32_exact,bf16,fp16",
                    help="extra precisions measured on the same frames at N=1 (',' separated; '' = none)")
    ap.add_argument("--plates", type=int, default=1, help="1: run YOLOv8n beside RetinaFace (BASELINE config 3)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--backend", default=os.environ.get("VD_DIST_BACKEND", "nccl"), choices=["nccl", "gloo"],
                    help="torch.distributed backend for N>1 (nccl = RCCL over xGMI; gloo for tests)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 (rehearsing the multi-rank path on a one-GPU box)")
    ap.add_argument("--records-out", default="", help="rank 0 saves the gathered box records of the last step (.npy)")
    ap.add_argument("--frames", type=int, default=0, help="strong scaling: total frames per step (default 64*8)")
    ap.add_argument("--option", action="append", default=[], help="name=value kernel-selection switch (vd_set_option)")
    ap.add_argument("--debug", action="append", default=[],
                    help="name=value timing-only experiment switch (vdt_set_debug; WRONG results while set)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip per-kernel HIP event timing")
    ap.add_argument("--inflight", type=int, default=1,
                    help="64-frame batches in flight: N contexts (own weights, streams, output and box buffers) take "
                         "consecutive steps round-robin, so one batch's letterbox / post / mosaic overlap another's convs")
    ap.add_argument("--microbatch", type=int, default=0, help="frames per depth-first backbone micro-batch (0: off)")
    ap.add_argument("--microbatch-stage", type=int, default=2, help="micro-batch the backbone through layer<N>")
    ap.add_argument("--faces", type=int, default=1, help="0: plates only, no mosaic (profiling the plate net)")
    ap.add_argument("--host-pipeline", type=int, default=1, help="1: also time the host-frame pipeline (PCIe incl.)")
    ap.add_argument("--force-dist", action="store_true",
                    help="process group + record all-gather even at one rank (exercises the RCCL branch at world 1)")
    ap.add_argument("--launch-probe", action="store_true",
                    help="each rank prints its rank / world as JSON and exits, no GPU work (launcher test)")
    return ap.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_cmd(argv, gpus, port):
    """The child command that starts `gpus` ranks of this script on one node (what the
    driver runs for N > 1): torch.distributed.run, 127.0.0.1 rendezvous."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(gpus),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def launch_ranks(argv, gpus):
    """Start the ranks as a child process (the parent has made no GPU call and is never
    replaced by exec) and return its exit status."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(launch_cmd(argv, gpus, _free_port()), env=env)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _oracle_pass(frames, m, ym, pri, bs, seconds):
    """Frames through the oracle `bs` at a time (one letterbox + forward per chunk, the
    per-frame post-processing and mosaic after it) until `seconds` have passed."""
    import torch
    from oracle import bbox, letterbox, mosaic
    from oracle.yolov8 import postprocess as yolo_post, raw_heads
    done, ref = 0, []
    t0 = time.perf_counter()
    while done < len(frames):
        chunk = list(frames[done:done + bs])
        x, _ = letterbox.preprocess(chunk)
        with torch.no_grad():
            loc, cls, _ = m.forward_raw(torch.from_numpy(x))
        if ym is not None:       # plate forward + NMS (boxes discarded like the reference)
            yx = letterbox.yolo_preprocess(chunk)
            with torch.no_grad():
                lv = ym(torch.from_numpy(yx))
            yolo_post(raw_heads(lv), [tuple(t.shape[2:]) for t in lv], yx.shape[2:], chunk[0].shape[:2])
        for i, img in enumerate(chunk):
            idx, boxes, _ = bbox.postprocess_frame(loc[i].numpy(), cls[i].numpy(), pri, 0.5, 0.4)
            ib = bbox.truncate_boxes(bbox.correct_and_scale(boxes, img.shape[0], img.shape[1]))
            mosaic.mosaic_frame(img, [tuple(int(v) for v in r) for r in ib], 8)
            ref.append((np.asarray(idx, np.int64), np.asarray(ib, np.int64).reshape(-1, 4)))
        done += len(chunk)
        if time.perf_counter() - t0 > seconds:
            break
    return done, time.perf_counter() - t0, ref


def cpu_baseline(frames, sd, seconds, plates=True, batch=8):
    """The CPU oracle on a bounded sample of the same synthetic frames, on this host's
    cores, doing what the headline step does per frame: torch-CPU fp32 RetinaFace +
    numpy decode/NMS/correction, the YOLOv8n plate forward + NMS beside it (when the
    headline runs plates; the reference discards plate boxes, combine_detect.py:239),
    and the sequential mosaic. Frames are forwarded `batch` at a time, as the
    reference batches its forwards (combine_detect.py:204,216; config.ini batch 64);
    the one-frame-at-a-time rate is kept as detail (`per_frame`). Returns the timing
    record and the oracle's per-frame (keep list, int boxes) for the parity block."""
    import torch
    from oracle import anchors
    from oracle.retinaface import build_oracle_model
    from oracle.yolov8 import build_oracle_yolo
    from vdmi import weights
    # the GPU box shares its host: use the per-GPU CPU share (OMP_NUM_THREADS, 16 there)
    cores = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    torch.set_num_threads(cores)
    m = build_oracle_model(sd)
    ym = build_oracle_yolo(weights.yolov8n_state_dict(0)) if plates else None
    pri = anchors.get_anchors((640, 640))
    _oracle_pass(frames[:batch], m, ym, pri, batch, 0.0)          # untimed: oneDNN primitive set-up
    _oracle_pass(frames[:1], m, ym, pri, 1, 0.0)
    done, dt, ref = _oracle_pass(frames, m, ym, pri, batch, seconds)
    d1, t1, _ = _oracle_pass(frames, m, ym, pri, 1, max(3.0, seconds / 3))
    what = (f"torch-CPU fp32 RetinaFace-R50 + numpy decode/NMS/mosaic"
            f"{' + YOLOv8n plate forward/NMS' if plates else ''}")
    rb, r1 = done / dt, d1 / t1
    # the baseline is the FASTER of the two forms (on 16 host cores one frame at a time
    # can beat 8-frame batches: the batch's activations leave the caches)
    best_b = rb >= r1
    form = (f"{batch} frames per forward (the reference batches its forwards, combine_detect.py:204,216)"
            if best_b else f"one frame per forward (faster here than {batch}-frame batches)")
    rec = {"value": max(rb, r1), "unit": "frames/s", "cores": cores, "kind": "port", "cpu_model": cpu_model(),
           "batch": batch if best_b else 1,
           "sample": f"{done if best_b else d1} x {frames.shape[2]}x{frames.shape[1]} synthetic frames through the "
                     f"oracle ({what}), {form}, {(dt if best_b else t1):.1f} s; the faster of the two forms",
           "batched": {"value": rb, "batch": batch, "frames": done, "seconds": round(dt, 2)},
           "per_frame": {"value": r1, "batch": 1, "frames": d1, "seconds": round(t1, 2)}}
    return rec, ref


def pmc_traffic(precision):
    """HBM bytes per face-conv launch (and per mosaic output pass) measured by the
    committed rocprofv3 PMC passes of this command at this precision
    (profiles/rNN_pmc_traffic*.json, tools/pmc_traffic.py); Nones when absent."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic*.json"))):
        d = json.load(open(f))
        if d.get("precision", "bf16") == precision:
            best = (d, f)
    if best is None:
        return None, None, None
    d, f = best
    blur = (d.get("mosaic_out_kernel") or {}).get("traffic_bytes_per_launch")
    return d.get("traffic_bytes_per_launch"), os.path.join("profiles", os.path.basename(f)), blur


def frame_lists(ctx, n):
    """Complete per-frame (anchor keep list, int boxes) of the last call."""
    from vdmi import _lib
    b = ctx.read_boxes(_lib.VD_NET_RETINAFACE, n)
    return [(b.label[i, :b.count[i]].astype(np.int64), b.xyxy[i, :b.count[i]].astype(np.int64)) for i in range(n)]


def agreement(a, b):
    """Fraction of frames whose keep lists (and int boxes) are identical."""
    n = min(len(a), len(b))
    if n == 0:
        return None, None
    keep = sum(np.array_equal(x[0], y[0]) for x, y in zip(a[:n], b[:n]))
    boxes = sum(np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]) for x, y in zip(a[:n], b[:n]))
    return round(keep / n, 4), round(boxes / n, 4)


class Mode:
    """One precision: its own context, the same frames, K timed steps."""

    def __init__(self, a, precision, dev, sd, plates):
        import vdmi
        from vdmi import _lib, weights
        opts = {k: int(v) for k, v in (o.split("=", 1) for o in a.option)}
        if precision == "fp32_exact":     # fp32 plan on exact-f32 MFMA
            opts["f32_split"] = 0
        if precision == "fp32_x6":        # fp32 plan on the exact 3-term bf16 split (6 products)
            opts["f32_split"] = 1
        self.ctx = vdmi.Context(device=dev.index or 0, precision=precision.split("_")[0],
                                max_batch=a.batch, options=opts, microbatch=a.microbatch,
                                microbatch_stage=a.microbatch_stage)
        for k, v in (o.split("=", 1) for o in a.debug):
            self.ctx.set_debug(k, int(v))
        self.ctx.load_weights(_lib.VD_NET_RETINAFACE, sd)
        if plates:
            self.ctx.load_weights(_lib.VD_NET_YOLOV8N, weights.yolov8n_state_dict(0))
        self.precision = precision
        self.face_groups = opts.get("face_groups", 2)   # runtime default (vd_common.h VdTune)
        self.faces = vdmi.DeviceBoxes(a.batch, 256, dev)
        self.pboxes = vdmi.DeviceBoxes(a.batch, 256, dev) if plates else None
        self.flags = _lib.VD_PROC_FACES | _lib.VD_PROC_MOSAIC | (_lib.VD_PROC_PLATES if plates else 0)
        if not a.faces:
            self.flags = _lib.VD_PROC_PLATES
        # --inflight N: slots 1..N-1 = further contexts, each on its own stream with its own
        # output frames and box lists; step i runs on slot i mod N (slot 0 = this context on
        # the caller's stream). `inflight` is how many take steps (the instrumented pass and
        # the host / JPEG legs use slot 0 alone).
        import torch
        self.torch = torch
        self.slots = []
        for _ in range(max(1, a.inflight) - 1):
            c = vdmi.Context(device=dev.index or 0, precision=precision.split("_")[0],
                             max_batch=a.batch, options=opts, microbatch=a.microbatch,
                             microbatch_stage=a.microbatch_stage)
            c.load_weights(_lib.VD_NET_RETINAFACE, sd)
            if plates:
                c.load_weights(_lib.VD_NET_YOLOV8N, weights.yolov8n_state_dict(0))
            st = torch.cuda.Stream(dev)
            c.set_stream(st.cuda_stream)
            self.slots.append((c, st, vdmi.DeviceBoxes(a.batch, 256, dev),
                               vdmi.DeviceBoxes(a.batch, 256, dev) if plates else None))
        self.inflight = 1 + len(self.slots)
        # with more than one slot, slot 0 runs on a stream of its own too: the caller's
        # (null) stream would serialise against the other slots' streams
        self.s0 = torch.cuda.Stream(dev) if self.slots else None
        self.s0_ready = False
        self.ready = [False] * len(self.slots)
        self.outs = {}
        self.step = 0
        self.cur = 0

    def next_slot(self, main):
        """The slot of the next step -> its torch stream (slot 0: `main`, this context's)."""
        k = self.step % self.inflight
        self.step += 1
        self.cur = k
        if k == 0:
            if self.s0 is not None and not self.s0_ready:
                self.s0.wait_stream(main)
                self.s0_ready = True
            return self.s0 or main
        st = self.slots[k - 1][1]
        if not self.ready[k - 1]:                 # once: the frames uploaded on `main` are visible
            st.wait_stream(main)
            self.ready[k - 1] = True
        return st

    def current(self, out):
        """(context, output frames, face boxes, plate boxes) of the current slot."""
        if self.cur == 0:
            return self.ctx, out, self.faces, self.pboxes
        c, st, fb, pb = self.slots[self.cur - 1]
        key = (self.cur, out.data_ptr(), tuple(out.shape))
        if key not in self.outs:
            with self.torch.cuda.stream(st):
                self.outs[key] = self.torch.empty_like(out)
        return c, self.outs[key], fb, pb

    def close(self):
        self.ctx.close()
        for c, *_ in self.slots:
            c.close()


def main():
    argv = sys.argv[1:]
    a = parse(argv)
    if a.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and (a.gpus > 1 or a.force_dist):
        # not started by torchrun: start the ranks now, before anything touches the GPU
        sys.exit(launch_ranks(argv, a.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}")
    if a.launch_probe:
        # one write(2) per line: the ranks share the parent's stdout pipe, and a line split
        # over two writes could interleave with another rank's
        sys.stdout.flush()
        os.write(1, (json.dumps({"rank": rank, "world": world, "local_rank": local}) + "\n").encode())
        return
    import torch
    import torch.distributed as dist
    from vdmi import _lib, synth, weights
    from vdmi.dist import RecordSink, process_frames, shard_range

    if a.same_device:
        local = 0
    dist_on = world > 1 or a.force_dist
    if dist_on:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")

    B, H, W = a.batch, a.height, a.width
    plates = bool(a.plates)
    sd = weights.retinaface_state_dict(0)
    # frames of this rank: weak = its own B frames; strong = its shard of one list
    if a.scaling == "strong":
        total = a.frames or B * 8
        f0, f1 = shard_range(total, world, rank)
        nloc = f1 - f0
        per_rank = -(-total // world)                    # records padded to the largest shard
    else:
        total = world * B
        f0, nloc, per_rank = rank * B, B, B
    batches = [(s, min(B, nloc - s)) for s in range(0, nloc, B)]
    # weak: this rank's own B distinct frames (hash frames f0 ..); strong: one list whose
    # frame g shows hash frame g mod B, whichever rank holds it (B distinct frames made
    # on the host once, the rank's whole shard gathered from them in HBM)
    start = f0 if a.scaling == "weak" else 0
    nhost = max(1, min(B, nloc if a.scaling == "weak" else total))
    if a.frames_src == "up2":
        host = np.repeat(np.repeat(synth.frames(nhost, H // 2, W // 2, seed=0, start=start), 2, axis=1), 2, axis=2)
    else:
        host = synth.frames(nhost, H, W, seed=0, start=start)
    frames = torch.from_numpy(host).to(dev)
    if a.scaling == "strong":
        frames = frames[torch.arange(f0, f0 + nloc, device=dev) % nhost].contiguous()
    out = torch.empty_like(frames)
    stream = torch.cuda.current_stream(dev)
    rec_cap = 64                      # box record: frame, count, 64 x (box, score, anchor)
    gathered = {}

    def run(mode, timed_steps, sync=True):
        for _ in range(timed_steps):
            with torch.cuda.stream(mode.next_slot(stream)):   # --inflight: this step's slot
                ctx, o, fb, pb = mode.current(out)
                # the product's shard loop (vdmi.dist.process_frames): one vd_process per batch,
                # each batch's box records packed on the context stream behind it
                sink = RecordSink(per_rank, cap=rec_cap, device=dev) if (dist_on or a.records_out) else None
                process_frames(ctx, frames, o, B, f0, sink, mode.flags, fb, pb)
                if dist_on:     # per-frame box records -> every rank (ONE RCCL all-gather over xGMI)
                    got = sink.gather()
                    if mode.precision == a.precision:
                        gathered["rec"] = got
                elif sink is not None and mode.precision == a.precision:
                    gathered["rec"] = sink.rec

    def timed(mode):
        torch.cuda.synchronize(dev)
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        run(mode, a.steps)
        torch.cuda.synchronize(dev)
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize(dev)
        d = time.perf_counter() - t0
        if dist_on:
            t = torch.tensor([d], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            d = float(t.item())
        return d

    def measure(precision):
        mode = Mode(a, precision, dev, sd, plates)
        mode.ctx.set_stream((mode.s0 or stream).cuda_stream)
        run(mode, a.warmup)
        # `value`: K steps with nothing but the work in the stream (no per-launch events)
        dt = timed(mode)
        res = {"value": round(total * a.steps / dt, 2), "ms_per_step": round(dt / a.steps * 1e3, 3)}
        if not a.no_timing:
            res.update(instrumented(mode, precision))
            rf = res["roofline"]
            # the timed steps' face-conv FLOPs over their whole wall time (every other
            # kernel of the step, the plate net included, counted against them)
            # is the headline figure: `achieved` / `frac` describe the timed
            # steps themselves; the per-launch figure of the face_groups=1 instrumented pass
            # (HIP events per launch, what the committed rocprof summaries check) is kept
            # under `per_launch`
            sa = rf["flop_per_step"] / (res["ms_per_step"] * 1e-3) / 1e12
            rf["per_launch"] = {k: rf[k] for k in ("achieved", "frac", "avg_launch_ms", "launches",
                                                   "flop_per_launch", "measured_with")}
            for k in ("avg_launch_ms", "launches", "flop_per_launch", "measured_with"):
                del rf[k]
            rf["achieved"], rf["frac"] = round(sa, 2), round(sa / rf["peak"], 4)
            rf["measured_with"] = (f"face-conv FLOP per step / ms_per_step of the timed steps (face_groups="
                                   f"{mode.face_groups}: every other kernel of the step, the plate net included, "
                                   "counted against the convs)")
        res["faces_per_frame"] = round(float(mode.faces.count.float().mean().item()), 2)
        lists = frame_lists(mode.ctx, batches[-1][1]) if batches and a.faces else []
        if world == 1 and precision == a.precision and a.host_pipeline:
            res["host_pipeline"] = host_pipeline(mode)
            res["jpeg_pipeline"] = jpeg_pipeline(mode)
            if (H, W) == (1080, 1920):   # realistic entropy: smooth structure + sensor noise, ~0.45 MB per q95 frame
                sf = synth.structured_frames(min(B, 8), H, W, seed=0)
                sf = np.concatenate([sf] * (-(-B // len(sf))))[:B]
                res["jpeg_pipeline_structured"] = jpeg_pipeline(mode, torch.from_numpy(sf).to(dev), "structured")
        mode.close()
        return res, lists

    def host_pipeline(mode):
        """The same workload from pinned HOST frames to pinned host output: H2D, the
        vd_process and the D2H of frames and box lists on three streams
        (vdmi.pipeline.FramePipeline), batch i's copies overlapping batch i+-1's
        compute. The frames sit in the pinned slots a decoder would write into."""
        from vdmi.pipeline import FramePipeline
        pipe = FramePipeline(mode.ctx, H, W, max_batch=B, plates=plates)
        for _ in range(pipe.depth):                       # both slots hold real frames
            pipe.next_input(B)[...] = host[:B]
            pipe.collect(pipe.submit_filled(B))
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        pending = None
        for _ in range(a.steps):
            pipe.next_input(B)
            cur = pipe.submit_filled(B)
            if pending is not None:
                pipe.collect(pending)
            pending = cur
        pipe.collect(pending)
        d = time.perf_counter() - t0
        pipe.close()
        mode.ctx.set_stream(stream.cuda_stream)
        return {"value": round(B * a.steps / d, 2), "unit": "frames/s", "ms_per_step": round(d / a.steps * 1e3, 3),
                "pcie_bytes_per_step": 2 * B * H * W * 3,
                "what": "pinned host frames -> H2D -> vd_process -> D2H of mosaicked frames + box lists, "
                        "copies and compute on separate streams (FramePipeline, depth 2)"}

    def jpeg_pipeline(mode, src=None, what="noise"):
        """Frame I/O included: B frames as in-memory JPEG files (q95
        4:2:0, what the reference's ffmpeg split and cv2.imwrite produce) ->
        vd_jpeg_decode (device entropy decode + HIP IDCT) into device frames ->
        vd_process -> vd_jpeg_encode (HIP FDCT + device Huffman coding) -> JPEG bytes in
        host memory, as batch_process_images' GPU codec path runs it
        (vdmi.pipeline.GpuJpegStages): decode, process and encode of consecutive
        batches in flight on three contexts, chained by events (no device-wide syncs)."""
        from vdmi.pipeline import GpuJpegStages
        ctx = mode.ctx
        ctx.set_stream(stream.cuda_stream)
        if src is None:
            src = frames[:B]
        jp = ctx.jpeg_encode(src, quality=95, subsampling=2)
        steps = max(1, min(a.steps, 8))
        copts = {k: int(v) for k, v in (o.split("=", 1) for o in a.option) if k.startswith(("jdec_", "jenc_"))}
        st = GpuJpegStages(ctx, B, mode.flags, quality=95, subsampling=2, codec_options=copts)
        outj = []
        done = lambda key, res, nf, npl: outj.__setitem__(slice(None), res[0][1])
        try:
            st.run(((s, lambda: jp, None) for s in range(3)), done)       # warm-up
            torch.cuda.synchronize(dev)
            for k in st.stats:
                st.stats[k] = 0.0
            st.serial_jobs = 0
            t0 = time.perf_counter()
            st.run(((s, lambda: jp, None) for s in range(steps)), done)
            d = time.perf_counter() - t0
            passes = st.dctx.jdec_passes()
        finally:
            st.close()
        ctx.set_stream(stream.cuda_stream)
        stg = {k: round(v / steps * 1e3, 2) for k, v in st.stats.items()}
        return {"value": round(B * steps / d, 2), "unit": "frames/s", "ms_per_step": round(d / steps * 1e3, 3),
                "frames": what, "stage_ms_per_step": stg, "decode_sync_passes": passes, "steps": steps,
                "serial_decode_jobs": st.serial_jobs,
                "jpeg_bytes_in_per_frame": int(np.mean([len(j) for j in jp])),
                "jpeg_bytes_out_per_frame": int(np.mean([len(j) for j in outj])),
                "what": "in-memory q95 4:2:0 JPEG frames -> GPU decode (device entropy decode + HIP IDCT, second "
                        "context) -> vd_process -> GPU encode (HIP FDCT + device Huffman coding, third context) -> "
                        "JPEG bytes in host memory; decode, process and encode of consecutive batches in flight, "
                        "chained by events (vdmi.pipeline.GpuJpegStages)"}

    def instrumented(mode, precision):
        """Per-kernel-family durations: the same K steps again, each launch bracketed
        by HIP events on the stream it runs on (runtime.cpp t_begin / t_end). The face
        net runs as one launch per layer over the whole batch here (face_groups = 1):
        with frame groups on concurrent streams each launch's events would also span
        the other groups' work. The timed steps' own rate is `roofline.step`."""
        ctx = mode.ctx
        ctx.set_option("face_groups", 1)
        ctx.timing(True)
        ctx.timing_reset()
        nin, mode.inflight, mode.step = mode.inflight, 1, 0   # slot 0 alone
        dt_ev = timed(mode)
        mode.inflight = nin
        ctx.set_option("face_groups", mode.face_groups)
        r = {"instrumented_ms_per_step": round(dt_ev / a.steps * 1e3, 3)}
        cms, cn, cflop = ctx.timing_read(_lib.FAM_CONV)
        mms, mn, mbytes = ctx.timing_read(_lib.FAM_MOSAIC)
        lms, _, _ = ctx.timing_read(_lib.FAM_LETTERBOX)
        pms, _, _ = ctx.timing_read(_lib.FAM_POST)
        oms, _, _ = ctx.timing_read(_lib.FAM_OTHER)
        yms, yn, yflop = ctx.timing_read(_lib.FAM_PLATE_CONV)
        cms6, _, _ = ctx.timing_read(_lib.FAM_MOSAIC_CELLS)
        ctx.timing(False)
        ach = cflop / (cms * 1e-3) / 1e12 if cms > 0 else 0.0
        traffic, tsrc, blur_traffic = pmc_traffic(precision)
        peak = PEAK_TFLOPS[precision]
        kern = ("conv_x6_kernel<..., 3> launches (f32 operands split exactly into 3 bf16 terms, 6 products on "
                "v_mfma_f32_16x16x32_bf16, f32 accumulate; peak = 2500/6)" if precision == "fp32_x6" else
                "stem_pool32_kernel + bottleneck32_kernel / bottleneck32p_kernel + chain32_kernel + conv_x6_kernel<..., 2> / "
                "conv_x6_halo_kernel / conv1x1_x6_kernel<..., 2> "
                "launches (f32 operands scaled per frame / per "
                "channel by powers of two and split into fp16 pairs, 3 products on v_mfma_f32_16x16x32_f16, f32 "
                "accumulate; peak = 2500/3)" if precision == "fp32" else
                "conv_igemm_kernel<float> launches (exact-f32 v_mfma_f32_16x16x4_f32)" if precision == "fp32_exact" else
                "stem_pool + bottleneck (fused layer1) + chain (layer2) + conv_big + conv_igemm + conv1x1_stream "
                "launches on _Float16 operands" if precision == "fp16" else
                "stem_pool + bottleneck (fused layer1) + chain (layer2) + conv_big + conv_igemm + conv1x1_stream")
        r["roofline"] = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
                         "frac": round(ach / peak, 4), "traffic": traffic,
                         "kernel": f"RetinaFace conv family: {kern} of a step, face stream (the plate net runs "
                                   "concurrently on a second stream)",
                         "avg_launch_ms": round(cms / max(cn, 1), 4), "launches": cn,
                         "flop_per_launch": round(cflop / max(cn, 1)), "traffic_unit": "bytes per launch (HBM, PMC)",
                         "traffic_source": tsrc,
                         "measured_with": "face_groups=1 (one launch per layer over the batch, face stream)",
                         "flop_per_step": round(cflop / max(a.steps, 1))}
        # blur: algorithmic bytes per launch = 2*W*H*3 per frame (out-of-place, reference
        # new-array semantics). Default (option mosaic_fused=1): ONE launch, the output pass
        # computes its bands' cell colours itself, so kernel == family; with mosaic_fused=0
        # the family adds the cell-table kernel (box prep + walked cell colours)
        bach = mbytes / (mms * 1e-3) / 1e9 if mms > 0 else 0.0
        fach = mbytes / ((mms + cms6) * 1e-3) / 1e9 if mms > 0 else 0.0
        fused = cms6 == 0
        r["blur_roofline"] = {"bound": "hbm", "achieved": round(bach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                              "frac": round(bach / PEAK_HBM_GBS, 4), "avg_launch_ms": round(mms / max(mn, 1), 4),
                              "bytes_per_launch": round(mbytes / max(mn, 1)),
                              "kernel": "mosaic_out_kernel<FUSED>" if fused else "mosaic_out_kernel<false>",
                              "traffic": blur_traffic, "traffic_source": tsrc,
                              "family": {"kernels": "mosaic_out_kernel<FUSED> (one launch: band cells walked in "
                                                    "its prelude)" if fused else
                                                    "mosaic_cell_kernel + mosaic_out_kernel<false>",
                                         "achieved": round(fach, 1), "frac": round(fach / PEAK_HBM_GBS, 4),
                                         "avg_ms_per_step": round((mms + cms6) / max(mn, 1), 4)}}
        steps = max(a.steps, 1)
        if yn:
            r["plate_conv"] = {"achieved_tflops": round(yflop / (yms * 1e-3) / 1e12, 2), "launches": yn,
                               "avg_launch_ms": round(yms / yn, 4)}
        r["ms_breakdown_per_step"] = {"conv": round(cms / steps, 3), "plate_conv": round(yms / steps, 3),
                                      "mosaic": round((mms + cms6) / steps, 3), "letterbox": round(lms / steps, 3),
                                      "post": round(pms / steps, 3), "other": round(oms / steps, 3)}
        return r

    head, head_lists = measure(a.precision)
    res = {
        "metric": f"end-to-end detect+blur FPS on {W}x{H} frames",
        "value": head["value"], "unit": "frames/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": head["ms_per_step"], "higher_is_better": True, "scaling": a.scaling,
        "vs_baseline": None, "dtype": "fp32" if a.precision.startswith("fp32") else a.precision,
        "data": "synthetic (counter-hash frames" + (", 2x nearest-upsampled" if a.frames_src == "up2" else "") +
                ", seeded random weights)",
        "config": {"workload": f"RetinaFace-R50+FPN+SSH{' + YOLOv8n plates' if plates else ''} detect + mosaic "
                               f"write-back, {total} frames of {W}x{H} per step over {world} GPU(s) "
                               f"(batches of {B} per GPU)",
                   "global_batch": total, "frame": f"{W}x{H}", "net_input": "640x640",
                   "parallelism": f"frame-sharded x{world}" + (
                       f", {'RCCL' if a.backend == 'nccl' else 'gloo'} all-gather of box records" if dist_on else ""),
                   "plates": plates, "batches_in_flight": max(1, a.inflight)},
    }
    for k in ("roofline", "blur_roofline", "faces_per_frame", "instrumented_ms_per_step", "plate_conv",
              "ms_breakdown_per_step", "host_pipeline", "jpeg_pipeline", "jpeg_pipeline_structured"):
        if k in head:
            res[k] = head[k]
    parity = {}
    mode_lists = {}
    if world == 1:
        modes = {}
        for p in [x for x in a.compare.split(",") if x and x != a.precision]:
            m, lists = measure(p)
            mode_lists[p] = lists
            keep, boxes = agreement(lists, head_lists)
            parity[f"{p}_vs_{a.precision}"] = {"keep_lists": keep, "int_boxes": boxes, "frames": len(lists)}
            m["parity_vs_" + a.precision] = parity[f"{p}_vs_{a.precision}"]
            modes[p] = {k: m[k] for k in ("value", "ms_per_step", "roofline", "parity_vs_" + a.precision,
                                          "faces_per_frame") if k in m}
            if "roofline" in modes[p]:
                modes[p]["roofline"] = {k: modes[p]["roofline"][k] for k in ("achieved", "peak", "frac",
                                                                             "per_launch")}
        if modes:
            res["modes"] = modes
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        base, ref = cpu_baseline(host[:64], sd, a.cpu_baseline_seconds, plates=plates)
        res["cpu_baseline"] = base
        for p, lists in [(a.precision, head_lists)] + list(mode_lists.items()):
            if p.startswith("fp32"):
                keep, boxes = agreement(lists, ref)
                parity[f"{p}_vs_oracle"] = {"keep_lists": keep, "int_boxes": boxes, "frames": len(ref)}
    if parity:
        parity["definition"] = ("fraction of bench frames whose complete keep lists (anchor indices in NMS "
                                "order) / keep lists and int boxes are identical")
        res["parity"] = parity
    if rank == 0 and a.records_out and "rec" in gathered:
        np.save(a.records_out, gathered["rec"].cpu().numpy())
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
