#!/bin/bash
# round 4: partial shard reads staged in overlapping runs (C5 from a host store)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python scripts/prof_c5host.py > $O/prof_c5host.jsonl 2> $O/prof_c5host.err
rc=$?; echo "prof rc=$rc"; head -c 1200 $O/prof_c5host.jsonl; exit $rc
