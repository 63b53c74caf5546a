"""GpuJpegStages on the bench's 64 noise / structured 1080p frames: frames/s and host stage
times for decode_overlap True / False / "auto" (noise JPEG regression study).

    python tools/jpeg_exp.py [noise|structured] [steps] [modes: comma list of true,false,auto] [codec opts k=v,...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "video-desensitization_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import vdmi
    from vdmi import _lib, synth, weights
    from vdmi.pipeline import GpuJpegStages
    kind = sys.argv[1] if len(sys.argv) > 1 else "noise"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    B = 64
    fr = synth.frames(B, 1080, 1920, seed=0) if kind == "noise" else \
        np.concatenate([synth.structured_frames(8, 1080, 1920, seed=0)] * 8)
    ctx = vdmi.Context(device=0, precision="fp32", max_batch=B)
    ctx.load_weights(_lib.VD_NET_RETINAFACE, weights.retinaface_state_dict(0))
    ctx.load_weights(_lib.VD_NET_YOLOV8N, weights.yolov8n_state_dict(0))
    flags = _lib.VD_PROC_FACES | _lib.VD_PROC_PLATES | _lib.VD_PROC_MOSAIC
    jp = ctx.jpeg_encode(torch.from_numpy(fr).cuda(), quality=95, subsampling=2)
    # process alone, for reference
    d = torch.from_numpy(fr).cuda()
    o = torch.empty_like(d)
    for _ in range(3):
        ctx.process(d, o, flags=flags)
    ctx.sync()
    t = time.perf_counter()
    for _ in range(steps):
        ctx.process(d, o, flags=flags)
    ctx.sync()
    print(f"{kind}: process alone {(time.perf_counter() - t) / steps * 1e3:.1f} ms/batch", flush=True)
    sel = (sys.argv[3] if len(sys.argv) > 3 else "true,false,auto").split(",")
    for mode in [{"true": True, "false": False, "auto": "auto"}[m] for m in sel]:
        copts = dict((k, int(v)) for k, v in (o.split("=") for o in sys.argv[4].split(","))) if len(sys.argv) > 4 else None
        st = GpuJpegStages(ctx, B, flags, quality=95, subsampling=2, decode_overlap=mode, codec_options=copts)
        try:
            st.run(((s, lambda: jp, None) for s in range(3)), lambda *a: None)
            torch.cuda.synchronize()
            for k in st.stats:
                st.stats[k] = 0.0
            t = time.perf_counter()
            st.run(((s, lambda: jp, None) for s in range(steps)), lambda *a: None)
            dt = time.perf_counter() - t
        finally:
            st.close()
        stg = {k: round(v / steps * 1e3, 1) for k, v in st.stats.items()}
        print(f"{kind} overlap={mode}: {B * steps / dt:.0f} frames/s, {dt / steps * 1e3:.1f} ms/batch, {stg}",
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
