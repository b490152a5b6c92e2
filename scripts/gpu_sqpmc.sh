#!/bin/bash
# SQ / GRBM counter passes (each its own run, kernel-trace only) over the
# headline bench command; TUNES = space-separated ablation bits to compare.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"; mkdir -p gpurun_out/sq
cd /tmp && export TMPDIR=/tmp
for tune in ${TUNES:-0}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d "$R/gpurun_out/sq/t$tune" -o pmc --output-format csv -- python "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --extra "" --tune $tune > "$R/gpurun_out/sq/t$tune.json" 2> "$R/gpurun_out/sq/t$tune.err"
  rc=$?; echo "sq pmc tune=$tune rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 "$R/gpurun_out/sq/t$tune.err"; exit $rc; fi
  python "$R/scripts/pmc_summary.py" "$R/gpurun_out/sq/t$tune" k_decode "$R/gpurun_out/sq/t$tune.summary.json" > /dev/null
  python -c "import json;d=json.load(open('$R/gpurun_out/sq/t$tune.summary.json'));print($tune, {k:round(v) for k,v in d['median_per_launch_KiB'].items()})"
done
