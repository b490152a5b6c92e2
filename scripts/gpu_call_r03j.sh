set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/xw2
CONFIG=headline TUNES=67108864,1140850688,268435456,1342177280 COPIES=0 ROUNDS=7 timeout -k 10 600 python scripts/graphbench.py > gpurun_out/xw2/hl.jsonl 2> gpurun_out/xw2/hl.err
rc=$?; echo "gb hl rc=$rc"; grep decode gpurun_out/xw2/hl.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/xw2/hl.err; exit $rc; }
exit 0
