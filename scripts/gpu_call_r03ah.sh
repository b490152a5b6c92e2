#!/bin/bash
# round 3: host-read fuzz stress -- 512 large host-sourced cases (slab pipeline)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03ah
ZARR_HIP_FUZZ_LARGE=512 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k test_random_host_reads_large > gpurun_out/r03ah/fuzz_large.log 2>&1
rc=$?; echo "fuzz large rc=$rc"; tail -6 gpurun_out/r03ah/fuzz_large.log
exit $rc
