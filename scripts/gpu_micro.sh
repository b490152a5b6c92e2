#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R="$(pwd)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python scripts/microbench.py > gpurun_out/micro.jsonl 2> gpurun_out/micro.err
rc=$?; echo "micro rc=$rc"; cat gpurun_out/micro.jsonl; tail -3 gpurun_out/micro.err
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "${PMC:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --pmc $PMC -d "$R/gpurun_out/pmc" -o pmc --output-format csv -- python "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/pmc_bench.json" 2> "$R/gpurun_out/pmc.err"
  rc=$?; echo "pmc rc=$rc"; tail -2 "$R/gpurun_out/pmc.err"
fi
exit $rc
