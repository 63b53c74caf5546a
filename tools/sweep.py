"""A/B sweep of runtime schedule knobs in ONE process (interleaved rounds).

    python tools/sweep.py [--batch 64] [--rounds 3] [--steps 5]
Prints ms/step (median, min) per variant for faces+mosaic on 1080p frames.
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-desensitization_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--variants", default="0:2,8:1,8:2,16:1,16:2,32:2")
    a = ap.parse_args()
    import torch
    import vdmi
    from vdmi import _lib, synth, weights
    dev = torch.device("cuda:0")
    B = a.batch
    frames = torch.from_numpy(synth.frames(B, 1080, 1920)).to(dev)
    out = torch.empty_like(frames)
    sd = weights.retinaface_state_dict(0)
    variants = [tuple(int(x) for x in v.split(":")) for v in a.variants.split(",")]
    ctxs = {}
    for mb, st in variants:
        c = vdmi.Context(max_batch=B, microbatch=mb, microbatch_stage=st)
        c.load_weights(_lib.VD_NET_RETINAFACE, sd)
        c.set_stream(torch.cuda.current_stream().cuda_stream)
        ctxs[(mb, st)] = (c, vdmi.DeviceBoxes(B, 256, dev))
    times = {k: [] for k in ctxs}
    for r in range(a.rounds + 1):
        for k, (c, fb) in ctxs.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                c.process(frames, out, faces=fb)
            torch.cuda.synchronize()
            if r:
                times[k].append((time.perf_counter() - t0) / a.steps * 1e3)
    for k, v in times.items():
        print(f"mb={k[0]:3d} stage={k[1]}  median {statistics.median(v):7.3f} ms  min {min(v):7.3f} ms  "
              f"({B / statistics.median(v) * 1e3:8.1f} fps)", flush=True)


if __name__ == "__main__":
    main()
