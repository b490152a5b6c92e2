#!/bin/bash
# round 4: k_encode_pair with the 11/11/10 pair tables vs the byte tables
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
ARMS="c2:0,c2:1,c2:0,c2:1,c3_64:0,c3_64:1,c3_64:2" timeout -k 10 400 python scripts/encbench.py > $O/enc_arms.jsonl 2> $O/enc_arms.err
rc=$?; echo "enc rc=$rc"; cat $O/enc_arms.jsonl; exit $rc
