#!/bin/bash
# round 3: the GPU suite on the library with k_decode_tile4f as an opt-in arm
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03ad
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03ad/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03ad/pytest.log
exit $rc
