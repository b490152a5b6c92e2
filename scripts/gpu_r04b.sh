#!/bin/bash
# round 4: full GPU suite (deferred CRC verdicts now in k_decode_il), the il
# publication arms, the self-launched 2-rank rehearsal, the cpp example leg,
# the uncached per-call profile
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
ARMS="prod=0:0,ret=0:1,tuned_nopub=1073741824:0,prod2=0:0" timeout -k 10 300 python scripts/armbench.py > $O/arms_headline.jsonl 2> $O/arms_headline.err
rc=$?; echo "arms rc=$rc"; cat $O/arms_headline.jsonl; [ $rc -ne 0 ] && { tail -5 $O/arms_headline.err; exit $rc; }
ZHIP_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --extra "" > $O/bench_rehearsal_2.json 2> $O/bench_rehearsal_2.err
rc=$?; echo "rehearsal rc=$rc"; cat $O/bench_rehearsal_2.json; tail -3 $O/bench_rehearsal_2.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --extra cpp,call > $O/bench_cpp.json 2> $O/bench_cpp.err
rc=$?; echo "bench cpp rc=$rc"; cat $O/bench_cpp.json; tail -3 $O/bench_cpp.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/prof_uncached.py > $O/prof_uncached.jsonl 2> $O/prof_uncached.err
rc=$?; echo "prof rc=$rc"; head -c 600 $O/prof_uncached.jsonl
[ $rc -ne 0 ] && exit $rc
for w in 8 1; do
  WORLD=$w timeout -k 10 200 python scripts/stamps.py > $O/stamps_il_w$w.jsonl 2> $O/stamps_il_w$w.err
  rc=$?; echo "stamps w=$w rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/stamps_il_w$w.err; exit $rc; }
done
for cfg in share8 share4 c3 c3g c4; do
  A="prod=0:0,ret=0:1,lean=16384:0"; case $cfg in c3*) A="prod=0:0,ret=0:2";; c4) A="prod=0:0,il=67108864:0,il_ret=67108864:1";; esac
  CONFIG=$cfg ARMS="$A" timeout -k 10 300 python scripts/armbench.py > $O/arms_$cfg.jsonl 2> $O/arms_$cfg.err
  rc=$?; echo "arms $cfg rc=$rc"; cat $O/arms_$cfg.jsonl; [ $rc -ne 0 ] && { tail -5 $O/arms_$cfg.err; exit $rc; }
done
exit $rc
