#!/bin/bash
# SQ counter pass over the encode-only harness (scripts/encbench.py), one run
# per TUNE value, kernel-trace only; summaries per kernel name (KERNELS:
# name substrings, e.g. "k_encode_pair<true k_encode_pair<false"; ENC_ARMS:
# encbench.py's ARMS).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"; mkdir -p gpurun_out/encsq
cd /tmp && export TMPDIR=/tmp
for tune in ${TUNES:-0}; do
  ARMS="${ENC_ARMS:-c3_64,c3_128}" TUNE=$tune STEPS=10 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT -d "$R/gpurun_out/encsq/t$tune" -o pmc --output-format csv -- python "$R/scripts/encbench.py" > "$R/gpurun_out/encsq/t$tune.json" 2> "$R/gpurun_out/encsq/t$tune.err"
  rc=$?; echo "enc sq pmc tune=$tune rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 "$R/gpurun_out/encsq/t$tune.err"; exit $rc; fi
  for k in ${KERNELS:-k_encode_tile4 k_encode_tileI}; do
    python "$R/scripts/pmc_summary.py" "$R/gpurun_out/encsq/t$tune" "$k" "$R/gpurun_out/encsq/t$tune.$k.json" > /dev/null
    python -c "import json;d=json.load(open('$R/gpurun_out/encsq/t$tune.$k.json'));print($tune, '$k', d['launches'].get('SQ_WAVE_CYCLES'), {k:round(v) for k,v in d['median_per_launch_KiB'].items()})"
  done
done
