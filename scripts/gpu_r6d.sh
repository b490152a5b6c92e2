#!/bin/bash
# Round 6: the mixed-spec write path and boundary fixes on the shipped library,
# the byte-table chain arms (66 / 67) on the tuning build, and their A/B on C3
# in 64^3 and 128^3 chunks.  Each GPU step under its own limit; stop at the
# first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r6d}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rectilinear.py tests/test_gpu_boundary.py \
  tests/test_gpu_multidevice.py tests/test_gpu_pipeline_suite.py -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > "$O/pytest_prod.log" 2>&1
rc=$?; echo "pytest prod rc=$rc"; tail -3 "$O/pytest_prod.log"; [ $rc -ne 0 ] && { tail -40 "$O/pytest_prod.log"; exit $rc; }
ZARR_HIP_ALLOW_LIB_OVERRIDE=1 ZHIP_LIB="$PWD/zarr-python_amd/zarr_hip/_lib/libzarrhip_tune.so" \
  timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_encode.py -m "gpu and tuning" -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "tilegw_and_tileg or tile4w_and_tile4 or 128_chunks or four_tile_form" > "$O/pytest_tune.log" 2>&1
rc=$?; echo "pytest tune rc=$rc"; tail -3 "$O/pytest_tune.log"; [ $rc -ne 0 ] && { tail -40 "$O/pytest_tune.log"; exit $rc; }
OUT=$O ROUNDS=15 CONFIGS="c3" ARMS="prod=0:0,bt=0:67,prod2=0:0,bt2=0:67" bash scripts/gpu_arms.sh || exit $?
OUT=$O ROUNDS=15 CONFIGS="c3g" ARMS="prod=0:0,bt=0:66,prod2=0:0,bt2=0:66" bash scripts/gpu_arms.sh || exit $?
ARMS="c3_128:0,c3_128:68,c3_128:0,c3_128:68" timeout -k 10 400 python scripts/encbench.py > "$O/enc_arms.jsonl" 2> "$O/enc_arms.err"
rc=$?; echo "enc rc=$rc"; cat "$O/enc_arms.jsonl"; [ $rc -ne 0 ] && { tail -5 "$O/enc_arms.err"; exit $rc; }
exit 0
