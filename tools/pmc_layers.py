"""Per-layer SQ counters of a `rocprofv3 --pmc ... --kernel-trace` run of bench.py
(faces only): maps the last step's conv dispatches onto the RetinaFace plan like
tools/conv_layers.py and prints, per layer, MFMA busy share and the wave-cycle
split (active / issue-stalled / parked at s_waitcnt or barrier).

    python tools/pmc_layers.py gpurun_out/pmc_sq/run_counter_collection.csv
"""
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_layers import face_plan  # noqa: E402

CONV = ("conv_igemm", "conv1x1_stream", "conv_big")


def main(path, B=64):
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        d = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]),
                                                    "t": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        d[r["Counter_Name"]] = float(r["Counter_Value"])
    ds = [d for _, d in sorted(disp.items())]
    plan = face_plan(B)
    stem_grid = (plan[0][1] + 127) // 128 * 256
    convs = [d for d in ds if any(k in d["name"] for k in CONV)]
    si = max(i for i, d in enumerate(convs) if d["grid"] == stem_grid)
    last = convs[si:si + len(plan)]
    print(f"{'layer':12s} {'us':>7s} {'mfma%':>6s} {'act%':>5s} {'istall%':>7s} {'park%':>6s} {'ldsconf':>8s}  kernel")
    for (name, M, N, K), d in zip(plan, last):
        wc = d.get("SQ_WAVE_CYCLES", 0) or 1
        busy = d.get("SQ_BUSY_CYCLES", 0) or 1
        kn = "big" if "conv_big" in d["name"] else ("stream" if "conv1x1" in d["name"] else "gemm")
        # SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over SIMDs; SQ_BUSY_CYCLES per SE-ish: report ratio raw
        print(f"{name:12s} {d['t'] / 1e3:7.1f} {100 * d.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / busy:6.1f} "
              f"{100 * d.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.1f} {100 * d.get('SQ_WAIT_INST_ANY', 0) / wc:7.1f} "
              f"{100 * d.get('SQ_WAIT_ANY', 0) / wc:6.1f} {d.get('SQ_LDS_BANK_CONFLICT', 0):8.0f}  {kn}")


if __name__ == "__main__":
    main(sys.argv[1])
