#!/bin/bash
# round 4: k_decode_tile4w (a wave per tile, one chain per lane) vs k_decode_tile4
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "tile4" > $O/pytest_tile4.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_tile4.log
[ $rc -ne 0 ] && exit $rc
CONFIG=c3 ARMS="prod=0:0,t4w=0:4,prod2=0:0,t4w2=0:4" timeout -k 10 300 python scripts/armbench.py > $O/arms_c3.jsonl 2> $O/arms_c3.err
rc=$?; echo "arms rc=$rc"; cat $O/arms_c3.jsonl; exit $rc
