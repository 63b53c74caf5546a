"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py into markdown:
per kernel (from the stats CSV) and per family (conv / mosaic / letterbox / post /
other), and — from the kernel trace next to it — the RetinaFace conv family on
its own stream (the plate network's convs run on a second stream), so the
per-launch averages can be checked against bench.py's in-process HIP-event
numbers (`roofline.avg_launch_ms` is the face conv family).

    python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv [out.md] [bench.json]

With bench.json (the same run's JSON line) the last `roofline.launches` face-stream
conv launches -- bench.py's instrumented pass, which runs last and issues the face net
as one launch per layer over the batch (face_groups = 1) -- are averaged on their own:
that is the number `roofline.avg_launch_ms` must agree with. The timed steps before it
run the face net as frame groups on two streams (both count as face streams).
"""
import json
import csv
import os
import sys

FAMILIES = [("conv", ("conv_igemm_kernel", "conv1x1_stream_kernel", "conv_big_kernel", "bottleneck_kernel",
                       "bottleneck32_kernel", "bottleneck32p_kernel", "stem_pool_kernel", "stem_pool32_kernel", "chain_kernel",
                       "chain32_kernel", "dwconv", "conv_x6_kernel", "conv_x6_halo_kernel",
                       "conv1x1_x6_kernel")),
            ("mosaic", ("mosaic_",)), ("letterbox", ("letterbox_kernel", "letterbox_s2d")),
            ("post", ("candidates_kernel", "nms_kernel")), ("other", ("maxpool", "upsample")),
            ("jpeg", ("jpeg_idct_kernel", "jpeg_color_kernel"))]
CONV = FAMILIES[0][1]


def family(name):
    return next((f for f, keys in FAMILIES if any(k in name for k in keys)), None)


FACE_ONLY = ("stem_pool_kernel", "stem_pool32_kernel", "bottleneck_kernel", "bottleneck32_kernel", "chain_kernel", "face_candidates_kernel")


def face_stream(rows):
    """Stream id(s) of the RetinaFace branch: the stream of the face-only kernels
    (fused stem / layer1 blocks / layer2 chain / face decode); failing those, the
    stream of the 640-row face letterbox (the plate canvas is letterboxed in
    space-to-depth form too in bf16, so that name alone no longer tells)."""
    face = {r["Stream_Id"] for r in rows if any(k in r["Kernel_Name"] for k in FACE_ONLY)}
    if not face:
        face = {r["Stream_Id"] for r in rows if "letterbox_s2d" in r["Kernel_Name"]}
    if not face:
        face = {r["Stream_Id"] for r in rows if "letterbox_kernel" in r["Kernel_Name"] and r["Grid_Size_Y"] == "640"}
    return face


def face_stream_convs(trace_path, last=0):
    """[count, total ns] of conv launches on the face stream(s), on the others, and of
    the last `last` face-stream launches by start time."""
    rows = sorted(csv.DictReader(open(trace_path)), key=lambda r: int(r["Start_Timestamp"]))
    face = face_stream(rows)
    f, o, tail = [0, 0], [0, 0], []
    for r in rows:
        if any(k in r["Kernel_Name"] for k in CONV):
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            acc = f if r["Stream_Id"] in face else o
            acc[0] += 1
            acc[1] += d
            if r["Stream_Id"] in face:
                tail.append(d)
    tail = tail[-last:] if last else []
    return f, o, [len(tail), sum(tail)]


def main(path, out=None, bench=None):
    rows = list(csv.DictReader(open(path)))
    lines = ["| family | kernel | calls | total ms | avg us |", "|---|---|---:|---:|---:|"]
    fam_tot = {}
    for r in rows:
        name = r["Name"]
        fam = family(name)
        if fam is None:
            continue
        calls, tot = int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6
        t = fam_tot.setdefault(fam, [0, 0.0])
        t[0] += calls
        t[1] += tot
        short = name.replace("(anonymous namespace)::", "").replace("_ZN12_GLOBAL__N_1", "")[:70]
        lines.append(f"| {fam} | `{short}` | {calls} | {tot:.3f} | {tot / calls * 1e3:.1f} |")
    lines.append("")
    lines.append("| family | calls | total ms | avg us per launch |")
    lines.append("|---|---:|---:|---:|")
    for fam, (c, t) in fam_tot.items():
        lines.append(f"| {fam} | {c} | {t:.3f} | {t / c * 1e3:.1f} |")
    trace = os.path.join(os.path.dirname(path), os.path.basename(path).replace("kernel_stats", "kernel_trace"))
    if os.path.exists(trace):
        last = 0
        if bench:
            line = [x for x in open(bench).read().splitlines() if x.startswith("{")][-1]
            roof = json.loads(line)["roofline"]
            last = int(roof.get("per_launch", roof).get("launches", 0))
        (fc, ft), (oc, ot), (lc, lt) = face_stream_convs(trace, last)
        lines.append("")
        lines.append("| conv launches by stream | calls | total ms | avg us per launch |")
        lines.append("|---|---:|---:|---:|")
        if fc:
            lines.append(f"| RetinaFace (face stream) | {fc} | {ft / 1e6:.3f} | {ft / fc / 1e3:.1f} |")
        if oc:
            lines.append(f"| YOLOv8n (plate stream) | {oc} | {ot / 1e6:.3f} | {ot / oc / 1e3:.1f} |")
        if lc:
            lines.append(f"| RetinaFace, bench.py's instrumented pass (last {lc}, face_groups = 1) | {lc} | "
                         f"{lt / 1e6:.3f} | {lt / lc / 1e3:.1f} |")
    txt = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None, sys.argv[3] if len(sys.argv) > 3 else None)
