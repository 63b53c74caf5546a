"""Effective shader clock per kernel from a rocprofv3 GRBM_GUI_ACTIVE pass
(/opt/skills/guides/MI355X_MICROARCH.md, DVFS give-back: clock ~= GRBM_GUI_ACTIVE / 8 /
kernel wall time, the counter summed over the 8 XCDs; reliable for dispatches of
>= 0.3 ms). Groups dispatches by kernel name and prints the duration-weighted clock.

    python tools/clock_pmc.py <rocprofv3 -d dir> [min_us]
"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 100.0
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    dur = {r["Dispatch_Id"]: (float(r["End_Timestamp"]) - float(r["Start_Timestamp"]), r["Kernel_Name"])
           for r in csv.DictReader(open(tr))}
    agg = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for r in csv.DictReader(open(cc)):
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE" or r["Dispatch_Id"] not in dur:
            continue
        ns, name = dur[r["Dispatch_Id"]]
        if ns < min_us * 1e3:
            continue
        a = agg[name.replace("void (anonymous namespace)::", "").split("(")[0][:70]]
        a[0] += float(r["Counter_Value"]) / 8.0
        a[1] += ns
        a[2] += 1
    tot = [0.0, 0.0]
    for k, (cyc, ns, n) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:70s} n={n:4d} {ns / 1e3 / n:9.1f} us  clock {cyc / ns:5.3f} GHz")
        tot[0] += cyc
        tot[1] += ns
    if tot[1]:
        print(f"all dispatches >= {min_us:.0f} us: duration-weighted clock {tot[0] / tot[1]:.3f} GHz")


if __name__ == "__main__":
    main()
