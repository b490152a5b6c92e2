#!/bin/bash
# round 4: per-call read host path (zhip_upload, raw pointers, item records)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/prof_uncached.py > $O/prof_uncached.jsonl 2> $O/prof_uncached.err
rc=$?; echo "prof rc=$rc"; head -c 1500 $O/prof_uncached.jsonl; exit $rc
