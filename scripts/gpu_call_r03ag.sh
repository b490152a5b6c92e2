#!/bin/bash
# round 3: seeded fuzz stress -- 10 000 further random cases (seeds 1660..11659)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03ag
ZARR_HIP_FUZZ_FIRST=1660 ZARR_HIP_FUZZ_SEEDS=10000 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k test_random_roundtrip > gpurun_out/r03ag/fuzz_stress.log 2>&1
rc=$?; echo "fuzz rc=$rc"; tail -8 gpurun_out/r03ag/fuzz_stress.log
exit $rc
