#!/bin/bash
# Round 6: the widest-interleave choice per config -- headline (S = 32 vs 8),
# C5's 512 KiB inner chunks (S = 16 vs 8), the C2 encode (S = 32 vs 8).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r6h}; mkdir -p "$O"
export TMPDIR=/tmp
ZARR_HIP_ALLOW_LIB_OVERRIDE=1 ZHIP_LIB="$PWD/zarr-python_amd/zarr_hip/_lib/libzarrhip_tune.so" \
  timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_configs.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$O/pytest.log"; [ $rc -ne 0 ] && { tail -40 "$O/pytest.log"; exit $rc; }
OUT=$O ROUNDS=15 CONFIGS="headline" ARMS="prod=0:0,s8=0:71,prod2=0:0,s8b=0:71,prod3=0:0,s8c=0:71" \
  bash scripts/gpu_arms.sh || exit $?
ARMS="c2:0,c2:73,c2:0,c2:73" timeout -k 10 400 python scripts/encbench.py > "$O/enc_arms.jsonl" 2> "$O/enc_arms.err"
rc=$?; echo "enc rc=$rc"; cat "$O/enc_arms.jsonl"; [ $rc -ne 0 ] && { tail -5 "$O/enc_arms.err"; exit $rc; }
ARMS="0,71,0,71" timeout -k 10 600 python scripts/c5_arms.py > "$O/c5_arms.jsonl" 2> "$O/c5_arms.err"
rc=$?; echo "c5 rc=$rc"; cat "$O/c5_arms.jsonl"; [ $rc -ne 0 ] && { tail -5 "$O/c5_arms.err"; exit $rc; }
exit 0
