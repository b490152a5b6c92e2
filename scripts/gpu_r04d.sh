#!/bin/bash
# round 4: line-spread returning publication (il, tile4) vs the round-3 and
# deferred arms; uncached per-call stage breakdown
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for cfg in headline share8 c3; do
  CONFIG=$cfg ARMS="prod=0:0,ret16=0:1,dv=0:2,prod2=0:0" timeout -k 10 300 python scripts/armbench.py > $O/arms_$cfg.jsonl 2> $O/arms_$cfg.err
  rc=$?; echo "arms $cfg rc=$rc"; cat $O/arms_$cfg.jsonl; [ $rc -ne 0 ] && { tail -5 $O/arms_$cfg.err; exit $rc; }
done
timeout -k 10 300 python scripts/prof_uncached.py > $O/prof_uncached.jsonl 2> $O/prof_uncached.err
rc=$?; echo "prof rc=$rc"; head -c 3000 $O/prof_uncached.jsonl; exit $rc
