#!/usr/bin/env python3
"""Per-kernel reduction of a rocprofv3 kernel trace of `bench.py`, with the single-stream profiled pass
separated from the two-stream timed steps.

bench.py runs W + K timed steps on two streams (the half-batch split: every launch covers half the batch,
launches of the two streams overlap, so their durations are not exclusive times) and then K profiled steps
on one stream (full-batch launches back to back, the pass its `roofline` is computed from).  In the trace the
profiled pass is the tail of the main queue after the side queue's last launch.  This prints, for that pass,
each kernel's launches, mean and total duration and ms per step, and the device-busy time per step; the same
for the whole trace; and writes both as JSON.

Usage: kt_reduce.py <kt_kernel_trace.csv> --steps K [--json out.json]
"""
import argparse
import collections
import csv
import json


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    i = n.find("(")
    return (n[:i] if i > 0 else n)[:110]


def reduce(rows, steps):
    acc = collections.OrderedDict()
    busy = 0
    for r in rows:
        k = short(r["Kernel_Name"]) + " grid=" + "x".join((r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"]))
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        e = acc.setdefault(k, [0, 0])
        e[0] += 1
        e[1] += d
        busy += d
    out = []
    for k, (n, ns) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
        out.append({"kernel": k, "launches": n, "mean_us": round(ns / n / 1e3, 3), "total_ms": round(ns / 1e6, 3),
                    "ms_per_step": round(ns / 1e6 / steps, 4) if steps else None})
    return out, busy


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True, help="profiled steps (bench.py --steps)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    queues = collections.Counter(r["Queue_Id"] for r in rows)
    main_q = queues.most_common(1)[0][0]
    side = [r for r in rows if r["Queue_Id"] != main_q]
    t_side = max(int(r["Start_Timestamp"]) for r in side) if side else 0
    prof = [r for r in rows if r["Queue_Id"] == main_q and int(r["Start_Timestamp"]) > t_side
            and "rocclr" not in r["Kernel_Name"]]
    res = {"trace": a.trace, "profiled_steps": a.steps, "main_queue": main_q, "queues": dict(queues)}
    if prof:
        span = (max(int(r["End_Timestamp"]) for r in prof) - min(int(r["Start_Timestamp"]) for r in prof)) / 1e6
        table, busy = reduce(prof, a.steps)
        res["single_stream_pass"] = {"launches": len(prof), "span_ms_per_step": round(span / a.steps, 4),
                                     "device_busy_ms_per_step": round(busy / 1e6 / a.steps, 4), "kernels": table}
        print(f"single-stream profiled pass: {len(prof)} launches, {span / a.steps:.3f} ms/step span, "
              f"{busy / 1e6 / a.steps:.3f} ms/step device-busy")
        for e in table[:40]:
            print(f"  {e['ms_per_step']:8.4f} ms/step  {e['launches']:5d} x {e['mean_us']:9.2f} us  {e['kernel']}")
    table, busy = reduce(rows, 0)
    res["whole_trace"] = {"launches": len(rows), "kernels": table}
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
