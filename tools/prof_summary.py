"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py into a markdown
table per kernel family (conv / mosaic / letterbox / post / other), so the
per-launch averages can be checked against bench.py's in-process HIP-event
numbers (roofline.avg_launch_ms).

    python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv [out.md]
"""
import csv
import sys

FAMILIES = [("conv", ("conv_igemm_kernel", "conv1x1_stream_kernel", "conv_big_kernel")), ("mosaic", ("mosaic_",)), ("letterbox", ("letterbox_kernel", "letterbox_s2d_kernel")),
            ("post", ("candidates_kernel", "nms_kernel")), ("other", ("maxpool", "upsample"))]


def main(path, out=None):
    rows = list(csv.DictReader(open(path)))
    lines = ["| family | kernel | calls | total ms | avg us |", "|---|---|---:|---:|---:|"]
    fam_tot = {}
    for r in rows:
        name = r["Name"]
        fam = next((f for f, keys in FAMILIES if any(k in name for k in keys)), None)
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
    txt = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
