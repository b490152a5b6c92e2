#!/bin/bash
# Round 6, first GPU session: the DF_WHOLE check and the look-back finalizer
# arms (tests on both libraries), then graph-timed A/B on the headline and the
# N = 8 / N = 4 shares.  Every GPU step under its own limit, stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6a; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "df_whole or whole_chunk" > "$O/pytest_prod.log" 2>&1
rc=$?; echo "pytest prod rc=$rc"; tail -2 "$O/pytest_prod.log"; [ $rc -ne 0 ] && exit $rc
ZARR_HIP_ALLOW_LIB_OVERRIDE=1 ZHIP_LIB="$PWD/zarr-python_amd/zarr_hip/_lib/libzarrhip_tune.so" \
  timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "lookback or split_publication or ilh_arm or df_whole" > "$O/pytest_tune.log" 2>&1
rc=$?; echo "pytest tune rc=$rc"; tail -2 "$O/pytest_tune.log"; [ $rc -ne 0 ] && exit $rc
OUT=$O ROUNDS=${ROUNDS:-15} CONFIGS="${CONFIGS:-headline share8 share4}" ARMS="${ARMS:-prod=0:0,lb=0:58,ilh=0:41,ilhlb=0:59}" \
  bash scripts/gpu_arms.sh
