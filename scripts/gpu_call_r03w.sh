#!/bin/bash
# round 3: GPU suite with the full-size C4 / C5 tests
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03w
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03w/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "full_size|passed|failed|Error" gpurun_out/r03w/pytest.log | tail -12
exit $rc
