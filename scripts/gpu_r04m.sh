#!/bin/bash
# round 4: k_encode_tile4w (arm 8) vs k_encode_tile4, C3 encode
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "tile4" > $O/pytest_enc.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_enc.log
[ $rc -ne 0 ] && exit $rc
ARMS="c3_64:0,c3_64:8,c3_64:0,c3_64:8" timeout -k 10 400 python scripts/encbench.py > $O/enc_arms.jsonl 2> $O/enc_arms.err
rc=$?; echo "enc rc=$rc"; cat $O/enc_arms.jsonl; exit $rc
