#!/usr/bin/env python
"""Recompute every bench line's HBM fraction from rocprofv3 kernel statistics
(measurement tool, round 6): the line's algorithmic bytes per launch (bench.py
extra.*.algorithmic_bytes) / the average duration rocprofv3 --kernel-trace
--stats reports for the kernel the line names, against 8 TB/s, next to the
bench's own event-timed fraction.

  python scripts/rocprof_table.py BENCH_JSON STATS_DIR OUT_JSON

STATS_DIR holds one rocprofv3 output tree per profiling run (scripts/
gpu_final.sh: the headline, and `bench.py --extra-only --extra X
--no-host-legs` for each group of config lines); each run's kernel trace is
matched to the lines of the run that produced it by the run's directory name
(hl, c1, c2, ...), and a line's kernel is taken over its largest-grid
dispatches (the full-batch launches the line times): the median duration
gives `rocprof_hbm_frac` (the bench's own kernel time is a median-like
statistic too: the smaller of the eager median and the graph span per launch),
the mean `rocprof_hbm_frac_mean`."""

import csv
import glob
import json
import os
import statistics
import sys

# bench label (zhip_last_kernel) -> the kernel's template name in rocprof
TEMPLATE = {
    "k_decode_il": "k_decode_il<", "k_decode_ilh": "k_decode_ilh<", "k_decode_ilw512": "k_decode_ilw<",
    "k_decode_lead": "k_decode_lead<", "k_decode_lead4": "k_decode_lead4<", "k_decode_lead8": "k_decode_lead4<",
    "k_decode_pair": "k_decode_pair<", "k_decode_duo": "k_decode_duo<", "k_decode": "k_decode<",
    "k_decode_tile2w": "k_decode_tile4w<", "k_decode_tile4w": "k_decode_tile4w<",
    "k_decode_tileg2w": "k_decode_tilegw<", "k_decode_tilegw": "k_decode_tilegw<",
    "k_encode_il": "k_encode_il<", "k_encode_tile2": "k_encode_tile4<", "k_encode_tile4": "k_encode_tile4<",
    "k_encode_tileg": "k_encode_tileg<", "k_encode_pair": "k_encode_pair<",
}
# bench line -> the profiling run (directory) that times it
RUN = {"headline": "hl", "c1_1d_bytes": "c1", "c2_unsharded_256": "c2", "sharded_default_chain_256": "c2",
       "c3_transpose_210": "c3", "c3_transpose_210_chunks128": "c3", "c4_sharded_1024": "c4",
       "c5_partial_2048": "c5", "encode_c2": "enc", "encode_c3": "enc", "encode_c3_chunks128": "enc",
       "cpp_example_4096": "cpp"}


def stats(stats_dir):
    """Per run: (kernel name, dispatches, average ns) of each kernel's LARGEST
    grid from the kernel trace (the full-batch launches the line times; the
    same kernel also runs smaller launches, e.g. slabs of host reads), else
    the kernel_stats summary."""
    out = {}
    for f in glob.glob(os.path.join(stats_dir, "**", "*kernel_trace.csv"), recursive=True):
        run = os.path.relpath(f, stats_dir).split(os.sep)[0]
        by = {}
        with open(f) as fh:
            for r in csv.DictReader(fh):
                g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
                by.setdefault(r["Kernel_Name"], {}).setdefault(g, []).append(
                    int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        out[run] = [(k, len(v[max(v)]), sum(v[max(v)]) / len(v[max(v)]), statistics.median(v[max(v)]))
                    for k, v in by.items()]
    for f in glob.glob(os.path.join(stats_dir, "**", "*kernel_stats.csv"), recursive=True):
        run = os.path.relpath(f, stats_dir).split(os.sep)[0]
        if run in out:
            continue
        with open(f) as fh:
            out[run] = [(r["Name"], int(r["Calls"]), float(r["AverageNs"]), float(r["AverageNs"]))
                        for r in csv.DictReader(fh)]
    return out


def main():
    bench_json, stats_dir, out_json = sys.argv[1:4]
    with open(bench_json) as fh:
        b = json.loads(fh.read().strip().splitlines()[-1])
    st = stats(stats_dir)
    lines = {"headline": {"kernel": b["roofline"]["kernel"].split("::")[1].split("<")[0],
                          "algorithmic_bytes": b["roofline"]["algorithmic_bytes_per_launch"],
                          "hbm_frac": b["roofline"]["frac"]}}
    for k, v in b.get("extra", {}).items():
        if isinstance(v, dict) and "algorithmic_bytes" in v and "kernel" in v:
            lines[k] = v
        elif k == "cpp_example_4096" and isinstance(v, dict) and "device_uncompressed" in v:
            lines[k] = v["device_uncompressed"]
    rows = []
    for name, v in lines.items():
        label = v["kernel"].split(" ")[0]
        tmpl = TEMPLATE.get(label)
        run = RUN.get(name)
        cand = [r for r in st.get(run, []) if tmpl and ("zhip::" + tmpl) in r[0]]
        if not cand:
            rows.append({"line": name, "kernel": label, "rocprof": None})
            continue
        nm, calls, avg, med = max(cand, key=lambda r: r[1] * r[2])  # the dominant instantiation
        frac = v["algorithmic_bytes"] / (med * 1e-9) / 8e12
        rows.append({"line": name, "kernel": label, "rocprof_kernel": nm[:160], "calls_largest_grid": calls,
                     "rocprof_avg_us": round(avg / 1e3, 3), "rocprof_median_us": round(med / 1e3, 3),
                     "algorithmic_bytes": v["algorithmic_bytes"],
                     "rocprof_hbm_frac": round(frac, 4),
                     "rocprof_hbm_frac_mean": round(v["algorithmic_bytes"] / (avg * 1e-9) / 8e12, 4),
                     "bench_hbm_frac": v["hbm_frac"], "rel_diff": round(frac / v["hbm_frac"] - 1.0, 4)})
    with open(out_json, "w") as fh:
        json.dump({"bench": os.path.basename(bench_json), "lib_sha16": b.get("roofline", {}).get("lib_sha16"),
                   "rows": rows}, fh, indent=1)
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
