"""GPU kernel time by stage (decode / process / encode) in a rocprofv3 --kernel-trace of
tools/jpeg_exp.py: per-family totals and busy time (union of intervals), and the busy
time of the three families together, over the last `steps` process calls.

    python tools/jpeg_kernels.py <rocprofv3 -d dir> [steps]
"""
import csv
import glob
import os
import sys


def fam(n):
    if "jdec" in n or "jpeg_idct" in n or "jpeg_color" in n or "jpeg_up" in n:
        return "decode"
    if "jpeg_fdct" in n or "jpeg_h" in n or "jpeg_stuff" in n or "jenc" in n:
        return "encode"
    return "process"


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if ce is not None else 0)


def main():
    d = sys.argv[1]
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0])
                  for r in csv.DictReader(open(tr)))
    # the overlapped run: from the first jdec kernel after the last "process alone" stretch
    lb = [r[0] for r in rows if "letterbox" in r[2]]
    enc = [r for r in rows if fam(r[2]) == "encode"]
    t0 = enc[len(enc) // 3][0] if enc else rows[0][0]     # skip the warm-up encodes
    t1 = rows[-1][1]
    sel = [r for r in rows if r[0] >= t0]
    span = t1 - t0
    print(f"window {span / 1e6:.2f} ms, {len(lb)} letterbox launches in the trace")
    per = {}
    for f in ("decode", "process", "encode"):
        iv = [(s, e) for s, e, n in sel if fam(n) == f]
        per[f] = iv
        tot = sum(e - s for s, e in iv)
        print(f"  {f:8s} launches {len(iv):5d} sum {tot / 1e6:8.2f} ms busy {union(iv) / 1e6:8.2f} ms")
    print(f"  all busy {union([x for v in per.values() for x in v]) / 1e6:.2f} ms")
    byname = {}
    for s, e, n in sel:
        if fam(n) != "process":
            byname.setdefault(n[:50], [0, 0])
            byname[n[:50]][0] += 1
            byname[n[:50]][1] += e - s
    for n, (c, t) in sorted(byname.items(), key=lambda kv: -kv[1][1])[:14]:
        print(f"    {n:50s} n={c:5d} {t / 1e6:8.2f} ms")


if __name__ == "__main__":
    main()
