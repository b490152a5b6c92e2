#!/bin/bash
# Round 6: the full GPU suite on the rebuilt libraries (the widest il
# interleave in production), then the headline A/B against the round-5
# interleave (arm 71, S = 8), then the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r6g}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$O/pytest_gpu.log"; cp gpurun_out/tuning_tests.log "$O/" 2>/dev/null
[ $rc -ne 0 ] && { tail -60 "$O/pytest_gpu.log"; tail -30 "$O/tuning_tests.log"; exit $rc; }
OUT=$O ROUNDS=15 CONFIGS="headline" ARMS="prod=0:0,s8=0:71,prod2=0:0,s8b=0:71" bash scripts/gpu_arms.sh || exit $?
timeout -k 10 700 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; tail -c 300 "$O/bench.json"; [ $rc -ne 0 ] && { tail -20 "$O/bench.err"; exit $rc; }
exit 0
