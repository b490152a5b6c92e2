#!/bin/bash
# Round 6 evidence on the shipped library: the full GPU suite and smoke, then
# scripts/gpu_final.sh (PMC traffic, the default bench line, rocprofv3 of the
# headline and of every config line, the rocprof fraction table), then a
# two-rank rehearsal of the N > 1 path on this one GPU (gloo; not a scaling
# number).  Stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/final}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$O/pytest_gpu.log"; cp gpurun_out/tuning_tests.log "$O/" 2>/dev/null
[ $rc -ne 0 ] && { tail -60 "$O/pytest_gpu.log"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$O/smoke.log"; [ $rc -ne 0 ] && exit $rc
OUT=$O bash scripts/gpu_final.sh || exit $?
ZHIP_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 --extra "" \
  --no-cpu-baseline > "$O/bench_rehearsal_2ranks.json" 2> "$O/bench_rehearsal_2ranks.err"
rc=$?; echo "rehearsal rc=$rc"; tail -c 300 "$O/bench_rehearsal_2ranks.json"
exit 0
