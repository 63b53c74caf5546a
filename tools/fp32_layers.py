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


def main(path, B=64, block=True, chain=2):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # fp32 plan: layer1 bottlenecks fused (block32.hip) unless option block_fuse32=0
    plan = face_plan(B, fused=True, block=block, chain={1: (0, 1, 2), 2: (0, 1, 2, 3, 4)} if chain == 1 else ({1: (0, 1, 2)} if chain == 2 else {}), ssh_fused=2, dual=(0,))
    # the face streams run the fused stem / layer1 kernels (with face_groups both group
    # streams do); the one with the latest launch is the context stream, which runs
    # bench.py's instrumented pass (face_groups = 1) last: its last len(plan) conv
    # launches are that pass's last step
    per = {}
    for r in rows:
        if "conv" in r["Kernel_Name"] or "stem_pool" in r["Kernel_Name"] or "bottleneck" in r["Kernel_Name"] \
                or "chain" in r["Kernel_Name"]:
            per.setdefault(r["Stream_Id"], []).append(r)
    face = [v for v in per.values() if any("stem_pool" in r["Kernel_Name"] for r in v)] or list(per.values())
    convs = max(face, key=lambda v: int(v[-1]["End_Timestamp"]))[-len(plan):]
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
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 64, (sys.argv[3] != "0") if len(sys.argv) > 3 else True,
         int(sys.argv[4]) if len(sys.argv) > 4 else 2)   # the plan's option chain (fp32: 2 = layer2 chains)
