#!/bin/bash
# round 4: publication placement arms (il), per-call pool, full bench snapshot
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for cfg in headline share8; do
  CONFIG=$cfg ARMS="prod=0:0,ret=0:1,ret_spread=0:3,nr_spread=0:4,plain_wg=0:5,nopub=1073741824:0,prod2=0:0" timeout -k 10 300 python scripts/armbench.py > $O/arms_$cfg.jsonl 2> $O/arms_$cfg.err
  rc=$?; echo "arms $cfg rc=$rc"; cat $O/arms_$cfg.jsonl; [ $rc -ne 0 ] && { tail -5 $O/arms_$cfg.err; exit $rc; }
done
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_full.json 2> $O/bench_full.err
rc=$?; echo "bench rc=$rc"; head -c 1500 $O/bench_full.json; tail -3 $O/bench_full.err
exit $rc
