set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/xw
ZHIP_TUNE=268435456 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/xw/pytest_xw.log 2>&1
rc=$?
echo "pytest (xw forced) rc=$rc"; tail -15 gpurun_out/xw/pytest_xw.log
if [ $rc -ne 0 ]; then exit $rc; fi
CONFIG=headline TUNES=134217728,67108864,268435456 COPIES=0 ROUNDS=7 timeout -k 10 600 python scripts/graphbench.py > gpurun_out/xw/hl.jsonl 2> gpurun_out/xw/hl.err
rc=$?; echo "gb hl rc=$rc"; grep -v scatterg_n gpurun_out/xw/hl.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/xw/hl.err; exit $rc; }
CONFIG=c4 TUNES=0,268435456 COPIES=0 ROUNDS=5 timeout -k 10 600 python scripts/graphbench.py > gpurun_out/xw/c4.jsonl 2> gpurun_out/xw/c4.err
rc=$?; echo "gb c4 rc=$rc"; grep -v scatterg_n gpurun_out/xw/c4.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/xw/c4.err; exit $rc; }
exit 0
