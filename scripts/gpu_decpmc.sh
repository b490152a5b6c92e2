#!/bin/bash
# SQ counter pass over the transposed-decode harness (scripts/tilebench.py), one run
# per TUNE value, kernel-trace only; summaries per kernel name.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"; mkdir -p gpurun_out/decsq
cd /tmp && export TMPDIR=/tmp
for tune in ${TUNES:-0}; do
  TUNE=$tune STEPS=10 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT -d "$R/gpurun_out/decsq/t$tune" -o pmc --output-format csv -- python "$R/scripts/tilebench.py" > "$R/gpurun_out/decsq/t$tune.json" 2> "$R/gpurun_out/decsq/t$tune.err"
  rc=$?; echo "dec sq pmc tune=$tune rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 "$R/gpurun_out/decsq/t$tune.err"; exit $rc; fi
  for k in k_decode_tile4 k_decode_tileg; do
    python "$R/scripts/pmc_summary.py" "$R/gpurun_out/decsq/t$tune" "$k" "$R/gpurun_out/decsq/t$tune.$k.json" > /dev/null
    python -c "import json;d=json.load(open('$R/gpurun_out/decsq/t$tune.$k.json'));print($tune, '$k', d['launches'].get('SQ_WAVE_CYCLES'), {k:round(v) for k,v in d['median_per_launch_KiB'].items()})"
  done
done
