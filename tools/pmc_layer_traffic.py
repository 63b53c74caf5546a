"""HBM traffic per RetinaFace layer from two rocprofv3 PMC passes of bench.py
(FETCH_SIZE / WRITE_SIZE with --kernel-trace; see tools/pmc_traffic.py for the
counter corrections): maps the last step's face conv launches onto the plan like
tools/conv_layers.py and prints per layer the measured bytes next to the
algorithmic bytes (inputs read once + outputs written once).

    python tools/pmc_layer_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write
"""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_layers import face_plan  # noqa: E402
from prof_summary import face_stream  # noqa: E402

KEYS = ("conv_igemm", "conv1x1_stream", "conv_big", "bottleneck_kernel", "stem_pool_kernel", "chain_kernel",
        "conv_persist")


def last_step(d, counter):
    trace = sorted(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))), key=lambda r: int(r["Start_Timestamp"]))
    vals = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    face = face_stream(trace)
    li = max(i for i, r in enumerate(trace) if r["Stream_Id"] in face and "letterbox" in r["Kernel_Name"])
    stream = trace[li]["Stream_Id"]
    rows = [r for r in trace[li:] if r["Stream_Id"] == stream and any(k in r["Kernel_Name"] for k in KEYS)]
    return [(vals.get(r["Dispatch_Id"], 0.0), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
            for r in rows]


def algo_bytes(name, M, N, K):
    if name.startswith("stem"):
        return 64 * 321 * 321 * 32 + M // 4 * 64 * 2
    if name.endswith(".block"):
        cin = 64 if name.startswith("l1.0") else 256
        return M * (cin + 256) * 2
    return None


def main(fd, wd):
    f = last_step(fd, "FETCH_SIZE")
    w = last_step(wd, "WRITE_SIZE")
    plan = face_plan(64)
    tot = 0.0
    print(f"{'layer':12s} {'us':>7s} {'read MB':>9s} {'write MB':>9s} {'TB/s':>6s}")
    for (name, M, N, K), (fk, t), (wk, _) in zip(plan, f, w):
        rb, wb = 2 * fk * 1024, wk * 1024
        tot += rb + wb
        print(f"{name:12s} {t:7.1f} {rb / 1e6:9.1f} {wb / 1e6:9.1f} {(rb + wb) / t / 1e6:6.2f}")
    print(f"total {tot / 1e9:.2f} GB")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
