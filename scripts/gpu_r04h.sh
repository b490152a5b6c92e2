#!/bin/bash
# round 4: k_decode_il with 16 blocks per lane (arm 3) vs production
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "il_arms or deferred" > $O/pytest_il.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_il.log
[ $rc -ne 0 ] && exit $rc
for cfg in headline share8 share4; do
  CONFIG=$cfg ARMS="prod=0:0,k16=0:3,prod2=0:0,k16b=0:3" timeout -k 10 300 python scripts/armbench.py > $O/arms_$cfg.jsonl 2> $O/arms_$cfg.err
  rc=$?; echo "arms $cfg rc=$rc"; cat $O/arms_$cfg.jsonl; [ $rc -ne 0 ] && { tail -5 $O/arms_$cfg.err; exit $rc; }
done
exit 0
