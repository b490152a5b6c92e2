#!/bin/bash
# round 4: k_decode_tile4w Horner placement arm (6), k_decode_tilegw arm (7), C3 / C3g
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "tileg or tile4" > $O/pytest_tile.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_tile.log
[ $rc -ne 0 ] && exit $rc
CONFIG=c3 ARMS="prod=0:0,early=0:6,tile4=0:5,prod2=0:0,early2=0:6" timeout -k 10 300 python scripts/armbench.py > $O/arms_c3.jsonl 2> $O/arms_c3.err
rc=$?; echo "arms rc=$rc"; cat $O/arms_c3.jsonl; [ $rc -ne 0 ] && { tail -5 $O/arms_c3.err; exit $rc; }
CONFIG=c3g ARMS="prod=0:0,gw=0:7,prod2=0:0,gw2=0:7" timeout -k 10 300 python scripts/armbench.py > $O/arms_c3g.jsonl 2> $O/arms_c3g.err
rc=$?; echo "arms c3g rc=$rc"; cat $O/arms_c3g.jsonl; [ $rc -ne 0 ] && { tail -5 $O/arms_c3g.err; exit $rc; }
exit 0
