set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sc4
CONFIG=headline TUNES=134217728,67108864 COPIES=0 ROUNDS=5 timeout -k 10 600 python scripts/graphbench.py > gpurun_out/sc4/hl.jsonl 2> gpurun_out/sc4/hl.err
rc=$?; echo "gb hl rc=$rc"; cat gpurun_out/sc4/hl.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/sc4/hl.err; exit $rc; }
CONFIG=c4 TUNES=0 COPIES=0 ROUNDS=5 timeout -k 10 600 python scripts/graphbench.py > gpurun_out/sc4/c4.jsonl 2> gpurun_out/sc4/c4.err
rc=$?; echo "gb c4 rc=$rc"; cat gpurun_out/sc4/c4.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/sc4/c4.err; exit $rc; }
exit 0
