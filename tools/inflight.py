"""Throughput with N vd_process batches in flight: N contexts (own weights, own
streams, own output and box buffers) take consecutive 64-frame steps round-robin,
so one batch's serial head (letterbox) and tail (post + mosaic) overlap another
batch's convs. Same synthetic frames and workload as bench.py's headline.

    python tools/inflight.py [--steps 20] [--warmup 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "video-desensitization_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--inflight", type=int, nargs="+", default=[1, 2])
    a = ap.parse_args()
    import vdmi
    from vdmi import _lib, synth, weights
    B, H, W = 64, 1080, 1920
    dev = torch.device("cuda:0")
    frames = torch.from_numpy(synth.frames(B, H, W, seed=0)).to(dev)
    sd, yd = weights.retinaface_state_dict(0), weights.yolov8n_state_dict(0)
    flags = _lib.VD_PROC_FACES | _lib.VD_PROC_MOSAIC | _lib.VD_PROC_PLATES
    res = {}
    for n in a.inflight:
        slots = []
        for i in range(n):
            ctx = vdmi.Context(device=0, precision="fp32", max_batch=B)
            ctx.load_weights(_lib.VD_NET_RETINAFACE, sd)
            ctx.load_weights(_lib.VD_NET_YOLOV8N, yd)
            st = torch.cuda.Stream(dev)
            ctx.set_stream(st.cuda_stream)
            slots.append((ctx, st, torch.empty_like(frames), vdmi.DeviceBoxes(B, 256, dev), vdmi.DeviceBoxes(B, 256, dev)))

        def run(k):
            for s in range(k):
                ctx, st, out, fb, pb = slots[s % n]
                ctx.process(frames, out, faces=fb, plates=pb, flags=flags)
        run(a.warmup * n)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        run(a.steps)
        torch.cuda.synchronize(dev)
        d = time.perf_counter() - t0
        ref = slots[0][2]
        same = all(torch.equal(s[2], ref) for s in slots[1:])
        res[f"inflight{n}"] = {"frames_per_s": round(B * a.steps / d, 1), "ms_per_step": round(d / a.steps * 1e3, 3),
                               "outputs_equal": same}
        print(json.dumps(res), flush=True)
        for s in slots:
            s[0].close()
        del slots
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
