#!/usr/bin/env python
"""Combine per-arm rocprofv3 --pmc summaries (scripts/gpu_arms_pmc.sh ->
profiles/r03/arms_pmc/<arm>.<pass>.summary.json) into one table per
workload with the derived ratios the round-3 review asked for:

  lds_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  wait_inst_frac    = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  wait_lds_frac     = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES
  tcc_hit_frac      = TCC_HIT / (TCC_HIT + TCC_MISS)
  ta_busy_frac      = TA_BUSY_avr / GRBM_GUI_ACTIVE

Counter values are per launch (median over the pass's launches); the
launches ran eagerly under counter collection, so their durations are not
timings -- the graph-timed microseconds come from scripts/graphbench.py and
are copied in from the jsonl given with --timing.

  python scripts/counters_table.py OUT.json ARM=LABEL ... [--timing f.jsonl ARM=ARMNAME ...]
"""
import json
import os
import sys

D = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r03", "arms_pmc")


def load(arm):
    row = {}
    for ps in ("sq", "insts", "mem"):
        f = os.path.join(D, f"{arm}.{ps}.summary.json")
        if os.path.exists(f):
            s = json.load(open(f))
            row.setdefault("kernels", s["kernels"])
            row.update({k: round(v) for k, v in s["median_per_launch_KiB"].items()})
    g = lambda k: float(row.get(k, 0.0))  # noqa: E731
    if g("SQ_LDS_IDX_ACTIVE"):
        row["lds_conflict_frac"] = round(g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE"), 3)
    if g("SQ_WAVE_CYCLES"):
        row["wait_inst_frac"] = round(g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES"), 3)
        row["wait_lds_frac"] = round(g("SQ_WAIT_INST_LDS") / g("SQ_WAVE_CYCLES"), 3)
    if g("TCC_HIT_sum") + g("TCC_MISS_sum"):
        row["tcc_hit_frac"] = round(g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum")), 3)
    if g("GRBM_GUI_ACTIVE") and g("TA_BUSY_avr"):
        row["ta_busy_frac"] = round(g("TA_BUSY_avr") / g("GRBM_GUI_ACTIVE"), 3)
    return row


def main():
    out, args = sys.argv[1], sys.argv[2:]
    timing, rest, arms = {}, [], {}
    if "--timing" in args:
        i = args.index("--timing")
        args, rest = args[:i], args[i + 1:]
    for a in args:
        k, v = a.split("=", 1)
        arms[v] = load(k)
        arms[v]["pmc_arm"] = k
    if rest:
        rows = {json.loads(line)["arm"]: json.loads(line) for line in open(rest[0]) if line.strip()}
        for a in rest[1:]:
            label, name = a.split("=", 1)
            timing[label] = rows[name]
    for label, t in timing.items():
        arms.setdefault(label, {})["graph_us_med"] = t["us_med"]
        arms[label]["graph_hbm_frac_min"] = t["hbm_frac_min"]
    json.dump({"source": "rocprofv3 --pmc, separate passes per counter group (scripts/gpu_arms_pmc.sh)",
               "arms": arms}, open(out, "w"), indent=1)
    print(json.dumps(arms, indent=1)[:3000])


if __name__ == "__main__":
    main()
