#!/usr/bin/env python
"""Summarise rocprofv3 --pmc passes (scripts/gpu_pmc.sh) into per-launch HBM
traffic for one kernel, corrected as MI355X_MICROARCH.md prescribes:
FETCH_SIZE (KiB) reports half the bytes of wide streaming reads on gfx950 ->
doubled; WRITE_SIZE (KiB) is exact for 16-byte-per-lane stores.

  python scripts/pmc_summary.py gpurun_out/pmc k_decode profiles/r01/pmc_traffic.json
"""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    pmc_dir, needle, out = sys.argv[1], sys.argv[2], sys.argv[3]
    vals: dict = {}
    names = set()
    for f in sorted(glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if needle not in row["Kernel_Name"]:
                    continue
                names.add(row["Kernel_Name"][:160])
                key = (row["Counter_Name"], row["Dispatch_Id"])
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    per: dict = {}
    for (ctr, _), v in vals.items():
        per.setdefault(ctr, []).append(v)
    med = {k: statistics.median(v) for k, v in per.items()}
    fetch = med.get("FETCH_SIZE")
    write = med.get("WRITE_SIZE")
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zarr-python_amd",
                       "zarr_hip", "_lib", "libzarrhip.so")
    try:
        import hashlib

        with open(lib, "rb") as fh:
            sha = hashlib.sha256(fh.read()).hexdigest()[:16]
    except OSError:
        sha = None
    res = {"kernel_match": needle, "kernels": sorted(names), "lib_sha16": sha,
           "launches": {k: len(v) for k, v in per.items()},
           "median_per_launch_KiB": med,
           "traffic_bytes_per_launch": None if fetch is None or write is None
           else int(round((2 * fetch + write) * 1024)),
           "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), WRITE_SIZE as reported; KiB"}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
