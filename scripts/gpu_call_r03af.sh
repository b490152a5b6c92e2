#!/bin/bash
# round 3: seeded fuzz stress -- further random cases (seeds 160..1659, then 1660..11659)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03af
ZARR_HIP_FUZZ_FIRST=160 ZARR_HIP_FUZZ_SEEDS=1500 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k test_random_roundtrip > gpurun_out/r03af/fuzz_stress.log 2>&1
rc=$?; echo "fuzz rc=$rc"; tail -15 gpurun_out/r03af/fuzz_stress.log
exit $rc
