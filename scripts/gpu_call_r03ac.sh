#!/bin/bash
# round 3: k_decode_tile4f (one A_64 chain per thread) -- tile tests, then
# graph-timed C3 against k_decode_tile4 (kTuneNoTile4F = bit 31), then the suite
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03ac
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "tile or transpose" > gpurun_out/r03ac/pytest_tile.log 2>&1
rc=$?; echo "pytest tile rc=$rc"; tail -25 gpurun_out/r03ac/pytest_tile.log; [ $rc -ne 0 ] && exit $rc
for tune in 0 -2147483648 0 -2147483648; do
  TUNE=$tune STEPS=20 ARMS=c3_64 timeout -k 10 200 python scripts/tilebench.py >> gpurun_out/r03ac/tilebench.jsonl 2>> gpurun_out/r03ac/tilebench.err
  rc=$?; echo "tilebench tune=$tune rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03ac/tilebench.err; exit $rc; }
done
cat gpurun_out/r03ac/tilebench.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03ac/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03ac/pytest.log
exit $rc
