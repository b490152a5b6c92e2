set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/xw3
CONFIG=c4 TUNES=0,268435456,1342177280,1073741824 COPIES=0 ROUNDS=5 timeout -k 10 600 python scripts/graphbench.py > gpurun_out/xw3/c4.jsonl 2> gpurun_out/xw3/c4.err
rc=$?; echo "gb c4 rc=$rc"; grep -v scatterg_n gpurun_out/xw3/c4.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/xw3/c4.err; exit $rc; }
exit 0
