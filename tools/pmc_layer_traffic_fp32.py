"""Per-layer HBM traffic of the fp32 face plan (conv-by-conv on conv_x6 /
conv1x1_x6) from two rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE with
--kernel-trace; corrections as tools/pmc_traffic.py): the last step's face conv
launches mapped onto face_plan(fused=False); per layer the measured bytes read
against the layer's input tensor (f32, M_in x Cin x 4 B; M_in = M x stride^2) --
the re-read factor -- and written against its output (M x N x 4 B).

    python tools/pmc_layer_traffic_fp32.py gpurun_out/<run>/pmc_fetch gpurun_out/<run>/pmc_write [B]
"""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_layers import face_plan  # noqa: E402

STRIDE2 = ("stem7x7", "l2.0.c2", "l2.0.ds", "l3.0.c2", "l3.0.ds", "l4.0.c2", "l4.0.ds")


def last_step(d, counter, n):
    trace = sorted(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))), key=lambda r: int(r["Start_Timestamp"]))
    vals = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    per = {}
    for r in trace:
        if "conv" in r["Kernel_Name"] or "stem_pool" in r["Kernel_Name"]:
            per.setdefault(r["Stream_Id"], []).append(r)
    rows = max(per.values(), key=len)[-n:]          # the face stream: most conv launches
    return [(vals.get(r["Dispatch_Id"], 0.0) * 1024.0, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
            for r in rows]


def main(fd, wd, B=64):
    plan = face_plan(B, fused=True, block=False, chain=False, ssh_fused=True, dual=(0,))
    f = last_step(fd, "FETCH_SIZE", len(plan))
    w = last_step(wd, "WRITE_SIZE", len(plan))
    print(f"{'layer':12s} {'us':>7s} {'read MB':>9s} {'in MB':>8s} {'reread':>6s} {'write MB':>9s} {'out MB':>8s}")
    for (name, M, N, K), (fb, t), (wb, _) in zip(plan, f, w):
        taps = 49 if name.startswith("stem") else (9 if K % 9 == 0 and K > 256 and not name.endswith(("c1", "c3", "ds"))
                                                   and not name.startswith(("fpn.o", "head")) else 1)
        cin = K // taps
        m_in = M * (4 if name in STRIDE2 else 1)
        in_b, out_b = m_in * cin * 4.0, M * N * 4.0
        rd = 2.0 * fb                                  # gfx950 FETCH_SIZE counts 128-B requests at 64 B
        print(f"{name:12s} {t:7.1f} {rd / 1e6:9.1f} {in_b / 1e6:8.1f} {rd / in_b:6.2f} {wb / 1e6:9.1f} {out_b / 1e6:8.1f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 64)
