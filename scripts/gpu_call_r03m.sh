set -u
cd "$GRAFT_REPO_ROOT"
ARMS="c4:0 c4:1 c4:64 copy:0:SIZE=4294967296,SPAN=4096,K=1,NT=3" PASSES="sq mem" bash scripts/gpu_arms_pmc.sh || exit $?
mkdir -p gpurun_out/c4p
CONFIG=c4 TUNES=0,1,64 COPIES=0 ROUNDS=3 timeout -k 10 600 python scripts/graphbench.py > gpurun_out/c4p/c4.jsonl 2> gpurun_out/c4p/c4.err
rc=$?; echo "gb c4 rc=$rc"; grep -v scatterg_ gpurun_out/c4p/c4.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/c4p/c4.err; exit $rc; }
exit 0
