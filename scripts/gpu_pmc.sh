#!/bin/bash
# PMC passes (each counter group its own run, kernel-trace only), per the guide,
# over the headline bench command (no extras, no CPU baseline); then the
# per-launch traffic summary of the decode kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"; mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_PMC:-}; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc ${grp//,/ } -d "$R/gpurun_out/pmc/p$i" -o pmc --output-format csv -- python "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --extra "" > "$R/gpurun_out/pmc/p$i.json" 2> "$R/gpurun_out/pmc/p$i.err"
  rc=$?; echo "pmc $grp rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python "$R/scripts/pmc_summary.py" "$R/gpurun_out/pmc" k_decode "$R/gpurun_out/pmc/pmc_traffic.json"
