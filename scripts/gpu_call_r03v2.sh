#!/bin/bash
# round 3: zarr v2 scenarios (V2Codec mapping), then the whole GPU suite
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03v2
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline_suite.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k v2 > gpurun_out/r03v2/pytest_v2.log 2>&1
rc=$?; echo "pytest v2 rc=$rc"; tail -30 gpurun_out/r03v2/pytest_v2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03v2/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03v2/pytest.log
exit $rc
