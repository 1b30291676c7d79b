#!/usr/bin/env python3
"""Two-stream overlap of a rocprofv3 kernel trace of `bench.py --no-profile` (round-5 analysis tool).

For the timed region (from the first side-queue launch to the last launch): wall time, time with no kernel
running, with one queue busy and with both busy; and per kernel name the summed durations.
Usage: kt_overlap.py <kt_kernel_trace.csv> --steps K
"""
import argparse
import collections
import csv

from kt_reduce import short


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"
            and "rocclr" not in r["Kernel_Name"]]
    qs = collections.Counter(r["Queue_Id"] for r in rows)
    if len(qs) < 2:
        print("single queue")
    side = [r for r in rows if r["Queue_Id"] != qs.most_common(1)[0][0]]
    t0 = min(int(r["Start_Timestamp"]) for r in side)
    sel = [r for r in rows if int(r["End_Timestamp"]) > t0]
    ev = []
    for r in sel:
        s, e = max(int(r["Start_Timestamp"]), t0), int(r["End_Timestamp"])
        ev.append((s, 1, r["Queue_Id"]))
        ev.append((e, -1, r["Queue_Id"]))
    ev.sort()
    busy = collections.Counter()
    cur = collections.Counter()
    last = t0
    for t, d, q in ev:
        n = sum(1 for v in cur.values() if v > 0)
        busy[n] += t - last
        last = t
        cur[q] += d
    wall = last - t0
    K = a.steps
    print(f"timed region: {wall / 1e6 / K:.3f} ms/step wall; idle {busy[0] / 1e6 / K:.3f}, one queue "
          f"{busy[1] / 1e6 / K:.3f}, both {sum(v for k, v in busy.items() if k >= 2) / 1e6 / K:.3f} ms/step")
    per = collections.Counter()
    for r in sel:
        per[short(r["Kernel_Name"])] += int(r["End_Timestamp"]) - max(int(r["Start_Timestamp"]), t0)
    for k, v in per.most_common(16):
        print(f"  {v / 1e6 / K:7.3f} ms/step  {k}")


if __name__ == "__main__":
    main()
