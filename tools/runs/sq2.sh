#!/bin/bash
# One rocprofv3 --pmc pass of MFMA-pipe / stall counters over the headline bench, per
# kernel name (mean per launch): MFMA busy share of the SIMD cycles, wave stall shares,
# LDS bank-conflict share. SQ_TAG names the output, SQ_FILTER a kernel-name regex.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
T=gpurun_out/${SQ_TAG:-sq2}
BARGS=${BARGS:-"--steps 2 --warmup 1 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing"}
mkdir -p $T
eval timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $T/a -o run --output-format csv -- python3 bench.py $BARGS > $T/a.log 2>&1 || { tail -5 $T/a.log; exit 1; }
python - <<PY
import csv, glob, re
from collections import defaultdict
flt = re.compile("${SQ_FILTER:-conv|bottleneck|stem}")
per = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
f = glob.glob("$T/a/**/*counter_collection.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    if not flt.search(k): continue
    per[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
out = []
for k in sorted(per):
    c = {x: v / max(len(n[k]), 1) for x, v in per[k].items()}
    busy = max(c.get("SQ_BUSY_CYCLES", 0), 1); wc = max(c.get("SQ_WAVE_CYCLES", 0), 1)
    # MFMA busy counts cycles summed over the SIMDs; SQ_BUSY_CYCLES per SE-quad -> report raw ratios too
    out.append(f"{k[:48]:48s} n={len(n[k]):3d} mfma_busy={c.get('SQ_VALU_MFMA_BUSY_CYCLES',0):.4g} sq_busy={busy:.4g} "
               f"gui={c.get('GRBM_GUI_ACTIVE',0):.4g} mfma_insts={c.get('SQ_INSTS_MFMA',0):.4g} "
               f"wait_any/wave={c.get('SQ_WAIT_ANY',0)/wc:.3f} wait_inst/wave={c.get('SQ_WAIT_INST_ANY',0)/wc:.3f} "
               f"bank_conf/lds={c.get('SQ_LDS_BANK_CONFLICT',0)/max(c.get('SQ_LDS_IDX_ACTIVE',0),1):.3f}")
open("$T/summary.txt", "w").write("\n".join(out) + "\n")
print("\n".join(out))
PY
