#!/usr/bin/env python3
"""Per-kernel mean counter values per dispatch from rocprofv3 --pmc csv output directories.
Usage: pmc_summary.py <dir> [<dir> ...] [--json out.json]"""
import csv
import glob
import json
import os
import sys


def collect(dirs):
    acc = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = row["Kernel_Name"]
                    c = row["Counter_Name"]
                    did = row.get("Dispatch_Id") or row.get("Correlation_Id")
                    e = acc.setdefault(k, {}).setdefault(c, {})
                    e[did] = e.get(did, 0.0) + float(row["Counter_Value"])
    out = {}
    for k, cs in acc.items():
        out[k] = {c: {"mean": sum(v.values()) / len(v), "n": len(v)} for c, v in cs.items()}
    return out


def main():
    args = sys.argv[1:]
    js = None
    if "--json" in args:
        i = args.index("--json")
        js = args[i + 1]
        args = args[:i] + args[i + 2:]
    res = collect(args)
    for k in sorted(res, key=lambda k: -res[k].get("SQ_WAVE_CYCLES", {"mean": 0})["mean"]):
        short = k.split("(")[0][-60:]
        print(short, {c: round(v["mean"], 1) for c, v in sorted(res[k].items())})
    if js:
        with open(js, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
