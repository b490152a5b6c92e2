#!/bin/bash
# SQ counter passes over the microbench (CRC pair kernel vs its CRC-free twin
# in one process); each pass its own kernel-trace-only run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"; mkdir -p gpurun_out/sqm
cd /tmp && export TMPDIR=/tmp
export ABLATIONS=0 ROUNDS=2
timeout -k 5 60 rocprofv3 -L > "$R/gpurun_out/sqm/avail.txt" 2>&1; echo "list rc=$?"
i=0
for set in "${PASSES[@]:-SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d "$R/gpurun_out/sqm/p$i" -o pmc --output-format csv -- python "$R/scripts/microbench.py" > "$R/gpurun_out/sqm/p$i.out" 2> "$R/gpurun_out/sqm/p$i.err"
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 "$R/gpurun_out/sqm/p$i.err"; exit $rc; fi
  for k in "k_decode_pair<true" "k_decode_pair<false"; do
    python "$R/scripts/pmc_summary.py" "$R/gpurun_out/sqm/p$i" "$k" "$R/gpurun_out/sqm/p$i.sum.json" | python -c "import json,sys;d=json.load(sys.stdin);print('$k', {a:round(b) for a,b in d['median_per_launch_KiB'].items()})"
  done
done
