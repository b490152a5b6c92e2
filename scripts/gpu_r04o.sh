#!/bin/bash
# round 4: encode publication words a line per chunk (production) vs 16 B apart (arm 9)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_all.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_all.log
[ $rc -ne 0 ] && exit $rc
ARMS="c2:0,c2:9,c3_64:0,c3_64:9,c2:0,c2:9,c3_64:0,c3_64:9" timeout -k 10 500 python scripts/encbench.py > $O/enc_arms.jsonl 2> $O/enc_arms.err
rc=$?; echo "enc rc=$rc"; cat $O/enc_arms.jsonl; exit $rc
