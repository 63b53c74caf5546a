"""HBM traffic per RetinaFace conv launch from two rocprofv3 PMC passes of the
same bench.py command (gfx950 slots do not fit FETCH_SIZE and WRITE_SIZE in one
pass; tools/gpu_run.sh `pmc`):

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write ...

Corrections (/opt/skills/guides/MI355X_MICROARCH.md § HBM): both counters are in
KiB; on gfx950 FETCH_SIZE tallies 128-B requests at 64 B, i.e. reports half of a
wide coalesced read, so bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024. Counters
also include Infinity-Cache hits. Face convs = conv dispatches on the face stream
(the stream of the face letterbox), matched to the counter rows by Dispatch_Id.

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write [out.json] [precision]
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import CONV, face_stream  # noqa: E402


def per_launch(d, counter):
    trace = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    face = face_stream(trace)
    ids = {r["Dispatch_Id"] for r in trace if r["Stream_Id"] in face and any(k in r["Kernel_Name"] for k in CONV)}
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv")))
            if r["Counter_Name"] == counter and r["Dispatch_Id"] in ids]
    return sum(vals) / max(len(vals), 1), len(vals)


def per_launch_named(d, counter, name):
    """Average counter per launch of the kernels whose name contains `name`."""
    trace = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    ids = {r["Dispatch_Id"] for r in trace if name in r["Kernel_Name"]}
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv")))
            if r["Counter_Name"] == counter and r["Dispatch_Id"] in ids]
    return sum(vals) / max(len(vals), 1), len(vals)


def main(fetch_dir, write_dir, out=None, precision="bf16"):
    f_kib, nf = per_launch(fetch_dir, "FETCH_SIZE")
    w_kib, nw = per_launch(write_dir, "WRITE_SIZE")
    mf, mnf = per_launch_named(fetch_dir, "FETCH_SIZE", "mosaic_out_kernel")
    mw, mnw = per_launch_named(write_dir, "WRITE_SIZE", "mosaic_out_kernel")
    res = {
        "precision": precision,
        "kernel": "RetinaFace conv launches on the face stream (" + ("stem_pool32 / bottleneck32 / conv_x6 / conv_x6_halo / conv1x1_x6, fp32 plan (scaled fp16 pairs)" if precision == "fp32"
                  else "stem_pool / bottleneck / chain / conv_big / conv_igemm / conv1x1_stream") + ")",
        "launches": {"fetch_pass": nf, "write_pass": nw},
        "fetch_size_kib_per_launch": round(f_kib, 1),
        "write_size_kib_per_launch": round(w_kib, 1),
        "traffic_bytes_per_launch": round((2.0 * f_kib + w_kib) * 1024.0),
        "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (KiB counters; gfx950 FETCH_SIZE = half of "
                      "wide coalesced reads); Infinity-Cache hits included",
        "mosaic_out_kernel": {"launches": {"fetch_pass": mnf, "write_pass": mnw},
                              "fetch_size_kib_per_launch": round(mf, 1), "write_size_kib_per_launch": round(mw, 1),
                              "traffic_bytes_per_launch": round((2.0 * mf + mw) * 1024.0)},
    }
    txt = json.dumps(res, indent=1)
    if out:
        open(out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None,
         sys.argv[4] if len(sys.argv) > 4 else "bf16")
