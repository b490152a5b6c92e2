#!/bin/bash
# Round 6: the full GPU suite on the rebuilt libraries, the default bench, and
# a rocprofv3 kernel-trace of the headline.  Each GPU step under its own limit,
# stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r6b}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$O/pytest_gpu.log"; cp gpurun_out/tuning_tests.log "$O/" 2>/dev/null
[ $rc -ne 0 ] && { tail -40 "$O/pytest_gpu.log"; exit $rc; }
timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; tail -c 600 "$O/bench.json"; [ $rc -ne 0 ] && { tail -20 "$O/bench.err"; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o hl -- python bench.py --steps 50 --extra "" \
  --no-cpu-baseline > "$O/bench_prof.json" 2> "$O/bench_prof.err"
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$O/bench_prof.err"; exit $rc; }
find "$O/prof" -name "*kernel_stats.csv" | head -3
exit 0
