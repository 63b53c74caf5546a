"""Per-layer view of the fp32 face plan (conv-by-conv) from a rocprofv3 kernel trace:
maps the last step's conv launches on the face stream onto face_plan(fused=False)
and prints duration, TFLOP/s and the kernel.

    python tools/fp32_layers.py gpurun_out/<dir>/run_kernel_trace.csv
"""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_layers import face_plan  # noqa: E402


def main(path, B=64, block=True):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # fp32 plan: layer1 bottlenecks fused (block32.hip) unless option block_fuse32=0
    plan = face_plan(B, fused=True, block=block, chain=False, ssh_fused=True, dual=(0,))
    # the face stream: the stream with the most conv launches (73 per step vs the plate net's 60);
    # its last len(plan) conv launches are the last step's layers
    per = {}
    for r in rows:
        if "conv" in r["Kernel_Name"] or "stem_pool" in r["Kernel_Name"] or "bottleneck" in r["Kernel_Name"]:
            per.setdefault(r["Stream_Id"], []).append(r)
    convs = max(per.values(), key=len)[-len(plan):]
    tot = fl_tot = 0
    for (name, M, N, K), r in zip(plan, convs):
        dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        fl = 2.0 * M * N * K
        tot += dt
        fl_tot += fl
        kn = r["Kernel_Name"].split("(")[0].replace("(anonymous namespace)::", "")[:40]
        grid = int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)
        print(f"{name:12s} M={M:8d} N={N:5d} K={K:5d} {dt*1e6:8.1f} us {fl/dt/1e12:7.1f} TF/s  wg={grid:6d} {kn}")
    print(f"total {tot*1e3:.2f} ms over {len(convs[:len(plan)])} launches, {fl_tot/tot/1e12:.1f} TF/s")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 64, (sys.argv[3] != "0") if len(sys.argv) > 3 else True)
