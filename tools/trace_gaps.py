#!/usr/bin/env python3
"""Busy time vs idle gaps between kernels over the last N steps of a rocprofv3 kernel trace.
A step starts at each launch of the marker kernel.  Usage: trace_gaps.py <kernel_trace.csv> [marker] [N]"""
import csv
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "conv0_moments"
nst = int(sys.argv[3]) if len(sys.argv) > 3 else 5
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
i0 = starts[-nst]
seg = rows[i0:]
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(seg, seg[1:])]
wall = int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])
print(f"steps {nst}: wall {wall / 1e6 / nst:.3f} ms/step, kernels busy {busy / 1e6 / nst:.3f}, "
      f"gaps {sum(g for g in gaps if g > 0) / 1e6 / nst:.3f} ({len(seg) / nst:.0f} launches/step, "
      f"median gap {sorted(gaps)[len(gaps) // 2] / 1e3:.1f} us)")
