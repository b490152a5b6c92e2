#!/bin/bash
# Bench + rocprof kernel stats only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-50}
timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 10 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${PROFILE:-1}" = "1" ]; then
  R="$GRAFT_REPO_ROOT"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python "$R/bench.py" --steps "$STEPS" --warmup 10 --no-cpu-baseline ${BENCH_ARGS:-} > "$R/gpurun_out/bench_prof.json" 2> "$R/gpurun_out/bench_prof.err"
  rc=$?; echo "rocprof rc=$rc"; cat "$R/gpurun_out/bench_prof.json"
  find "$R/gpurun_out/prof" -name "*stats*"
fi
exit $rc
