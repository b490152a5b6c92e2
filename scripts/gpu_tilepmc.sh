#!/bin/bash
# HBM traffic (FETCH_SIZE x2 + WRITE_SIZE, separate passes) of the transposed
# decodes in scripts/tilebench.py, per kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"; mkdir -p gpurun_out/tilepmc
cd /tmp && export TMPDIR=/tmp
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  STEPS=10 timeout -s KILL 120 rocprofv3 --pmc $grp -d "$R/gpurun_out/tilepmc/p$i" -o pmc --output-format csv -- python "$R/scripts/tilebench.py" > "$R/gpurun_out/tilepmc/p$i.json" 2> "$R/gpurun_out/tilepmc/p$i.err"
  rc=$?; echo "pmc $grp rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for k in k_decode_tile4 k_decode_tileg; do
  python "$R/scripts/pmc_summary.py" "$R/gpurun_out/tilepmc" "$k" "$R/gpurun_out/tilepmc/$k.json" > /dev/null
  python -c "import json;d=json.load(open('$R/gpurun_out/tilepmc/$k.json'));print('$k', d['traffic_bytes_per_launch'], d['launches'])"
done
