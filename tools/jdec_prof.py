"""Device JPEG decode alone: 64 synthetic 1080p q95 4:2:0 frames (noise or 4x-upsampled
'structured'), decoded into device memory N times; wall time per batch and passes.
Run under rocprofv3 --kernel-trace --stats for the per-kernel split.

    python tools/jdec_prof.py [noise|structured] [reps] [option=value ...]
"""
import io
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "video-desensitization_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402


def frames_jpeg(kind, n=64):
    from vdmi import synth
    fr = synth.frames(n, 1080, 1920, seed=3)
    if kind == "structured":
        fr = np.repeat(np.repeat(fr[:, ::4, ::4], 4, 1), 4, 2)
    out = []
    for f in fr:
        b = io.BytesIO()
        Image.fromarray(f).save(b, "JPEG", quality=95)
        out.append(b.getvalue())
    return out


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "noise"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    opts = {k: int(v) for k, v in (a.split("=") for a in sys.argv[3:])}
    import vdmi
    jp = frames_jpeg(kind)
    ctx = vdmi.Context(precision="fp32", max_batch=64, options=opts)
    d = torch.empty((64, 1080, 1920, 3), dtype=torch.uint8, device="cuda:0")
    ctx.jpeg_decode(jp, out=d)
    ctx.sync()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        ctx.jpeg_decode(jp, out=d)
        ctx.sync()
        ts.append(time.perf_counter() - t)
    print(f"{kind} {opts}: {np.mean([len(j) for j in jp]) / 1e6:.2f} MB/frame, decode {np.median(ts) * 1e3:.1f} ms "
          f"per 64 frames (min {min(ts) * 1e3:.1f}), passes {ctx.jdec_passes()}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
