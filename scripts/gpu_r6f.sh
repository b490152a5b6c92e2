#!/bin/bash
# Round 6: k_decode_il with interleave groups of 16 / 32 workgroups (tuning
# arms 69 / 70) -- exactness, then graph-timed A/B on the headline (twice).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r6f}; mkdir -p "$O"
export TMPDIR=/tmp
ZARR_HIP_ALLOW_LIB_OVERRIDE=1 ZHIP_LIB="$PWD/zarr-python_amd/zarr_hip/_lib/libzarrhip_tune.so" \
  timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m "gpu and tuning" -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "split_publication" > "$O/pytest_tune.log" 2>&1
rc=$?; echo "pytest tune rc=$rc"; tail -3 "$O/pytest_tune.log"; [ $rc -ne 0 ] && { tail -40 "$O/pytest_tune.log"; exit $rc; }
OUT=$O ROUNDS=15 CONFIGS="headline" ARMS="prod=0:0,s16=0:69,s32=0:70,prod2=0:0,s16b=0:69,s32b=0:70" \
  bash scripts/gpu_arms.sh || exit $?
exit 0
