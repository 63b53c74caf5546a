"""Per-stream timeline of the timed bench steps from a rocprofv3 --kernel-trace run of
bench.py (face frame groups on two streams, the plate net on a third):

    python tools/step_timeline.py <rocprofv3 -d dir> [steps_to_skip]

A step starts at a paired letterbox launch (face stream) and ends at the next one.
For each of the last full steps before bench.py's instrumented pass, prints per stream
its first start / last end / busy time (union of its kernel intervals) relative to the
step start, the time with 0 / 1 / 2 / 3+ kernels in flight, and the kernels running in
the step's last 2 ms (what the step's tail waits on).
"""
import csv
import glob
import os
import sys


def load(d):
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(tr)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"],
                     r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]))
    return sorted(rows)


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    rows = load(sys.argv[1])
    starts = [r[0] for r in rows if "letterbox_s2d_pair" in r[3] or "letterbox_s2d_lds_pair" in r[3]]
    if len(starts) < 3:
        starts = [r[0] for r in rows if "letterbox" in r[3]]
    plate_streams = {r[2] for r in rows if "yolo_candidates" in r[3]}
    face_streams = {r[2] for r in rows if "stem_pool" in r[3] or "bottleneck32" in r[3]}
    for k in range(max(0, len(starts) - 4), len(starts) - 2):   # skip the instrumented pass at the end
        t0, t1 = starts[k], starts[k + 1]
        step = [r for r in rows if t0 <= r[0] < t1]
        print(f"step {k}: {(t1 - t0) / 1e6:.3f} ms, {len(step)} launches")
        for st in sorted({r[2] for r in step}):
            iv = [(r[0], r[1]) for r in step if r[2] == st]
            tag = "plate" if st in plate_streams else ("face" if st in face_streams else "?")
            print(f"  stream {st:>3} {tag:5s} n={len(iv):3d} first {(min(s for s, _ in iv) - t0) / 1e6:7.3f} "
                  f"last end {(max(e for _, e in iv) - t0) / 1e6:7.3f} busy {union(iv) / 1e6:7.3f} ms")
        # concurrency histogram over [t0, t1)
        ev = sorted([(max(r[0], t0), 1) for r in step] + [(min(r[1], t1), -1) for r in step])
        hist, cur, last = [0, 0, 0, 0], 0, t0
        for t, d in ev:
            hist[min(cur, 3)] += t - last
            cur += d
            last = t
        hist[min(cur, 3)] += t1 - last
        print("  in flight 0/1/2/3+: " + " ".join(f"{h / 1e6:.3f}" for h in hist) + " ms")
        tail = [r for r in step if r[1] > t1 - 2_000_000]
        for r in tail[-14:]:
            print(f"    tail {(r[0] - t0) / 1e6:7.3f}-{(r[1] - t0) / 1e6:7.3f} s{r[2]:>3} {r[3][:60]}")


if __name__ == "__main__":
    main()
