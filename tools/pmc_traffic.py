#!/usr/bin/env python3
"""Fold the FETCH_SIZE / WRITE_SIZE passes of tools/pmc_traffic.sh into per-kernel HBM bytes per
launch.  FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes of wide
streaming reads (16 B/lane global_load and buffer_load ... lds alike), so it is doubled; WRITE_SIZE
is exact for 16-B stores (MI355X_MICROARCH.md "HBM").  Usage: pmc_traffic.py <outdir> <out.json> [bench args]"""
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                k = row["Kernel_Name"]
                e = acc.setdefault(k, {})
                did = row.get("Dispatch_Id") or row.get("Correlation_Id")
                e[did] = e.get(did, 0.0) + float(row["Counter_Value"])
    return {k: (len(v), sum(v.values())) for k, v in acc.items()}


def main():
    out, js = sys.argv[1], sys.argv[2]
    fetch = per_kernel(out, "FETCH_SIZE")
    write = per_kernel(out, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        nf, f = fetch.get(k, (0, 0.0))
        nw, w = write.get(k, (0, 0.0))
        n = max(nf, nw, 1)
        kernels[k] = {"launches": n, "fetch_bytes_per_launch": 2 * 1024 * f / max(nf, 1),
                      "write_bytes_per_launch": 1024 * w / max(nw, 1)}
        kernels[k]["hbm_bytes_per_launch"] = kernels[k]["fetch_bytes_per_launch"] + kernels[k]["write_bytes_per_launch"]
    res = {"note": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE (separate passes) over bench.py "
                   + " ".join(sys.argv[3:]) + "; FETCH_SIZE x2 (gfx950 correction), KiB -> bytes",
           "kernels": kernels}
    with open(js, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: round(v["hbm_bytes_per_launch"] / 1e6, 2) for k, v in kernels.items()}))


if __name__ == "__main__":
    main()
