"""Per-kernel SQ counter summary of two rocprofv3 --pmc passes (tools/g54.sh):
per kernel name, launches and the mean of each counter per launch, plus derived
ratios (waits / active issue per wave cycle; VALU and LDS instructions per MFMA).

    python tools/sq_summary.py gpurun_out/g54/sq gpurun_out/g54/sq2 [out.txt]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    per = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k].add(r["Dispatch_Id"])
    return per, n


def main(a, b, out=None):
    lines = []
    for d in (a, b):
        per, n = load(d)
        for k in sorted(per, key=lambda x: -len(n[x])):
            if not any(s in k for s in ("conv", "stem_pool")):
                continue
            c = {name: v / max(len(n[k]), 1) for name, v in per[k].items()}
            extra = ""
            if "SQ_INSTS_MFMA" in c and c["SQ_INSTS_MFMA"]:
                extra = " valu/mfma=%.2f lds/mfma=%.2f" % (c.get("SQ_INSTS_VALU", 0) / c["SQ_INSTS_MFMA"],
                                                         c.get("SQ_INSTS_LDS", 0) / c["SQ_INSTS_MFMA"])
            if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
                extra += " wait_any/wave=%.3f active/wave=%.3f" % (c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"],
                                                                   c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"])
            lines.append(f"{k[:48]:48s} n={len(n[k]):3d} " +
                         " ".join(f"{name}={v:.3g}" for name, v in sorted(c.items())) + extra)
        lines.append("")
    text = "\n".join(lines)
    print(text)
    if out:
        open(out, "w").write(text + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:4])
