"""Per-launch view of the fp32 plate net (YOLOv8n) from a rocprofv3 kernel trace of a
plates-only bench run (bench.py --faces 0): the launches of the last step between the
previous step's yolo_candidates_kernel and this step's, in launch order, with
duration, grid and kernel.

    python tools/plate_layers.py gpurun_out/<dir>/run_kernel_trace.csv
"""
import csv
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "yolo_candidates" in r["Kernel_Name"]]
    if len(ends) < 2:
        sys.exit("need two steps with yolo_candidates_kernel in the trace")
    step = rows[ends[-2] + 1:ends[-1]]
    tot = 0.0
    busy0, busy1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    for i, r in enumerate(step):
        dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
        tot += dt
        grid = int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1) * int(r.get("Grid_Size_Y", 1) or 1) \
            * int(r.get("Grid_Size_Z", 1) or 1)
        kn = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")[:70]
        print(f"{i:3d} {dt:8.1f} us wg={grid:6d} {kn}")
    print(f"total {tot / 1e3:.3f} ms of kernels over {len(step)} launches, span {(busy1 - busy0) * 1e-6:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
