set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/il2
ZHIP_TUNE=335544320 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/il2/pytest_ilvalu.log 2>&1
rc=$?
echo "pytest (il valu forced) rc=$rc"; tail -3 gpurun_out/il2/pytest_ilvalu.log
if [ $rc -ne 0 ]; then exit $rc; fi
CONFIG=c4 TUNES=0,134217728,67108864,335544320 ROUNDS=5 timeout -k 10 600 python scripts/graphbench.py > gpurun_out/il2/c4.jsonl 2> gpurun_out/il2/c4.err
rc=$?; echo "gb c4 rc=$rc"; grep decode gpurun_out/il2/c4.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/il2/c4.err; exit $rc; }
CONFIG=headline TUNES=134217728,67108864,335544320 ROUNDS=5 timeout -k 10 600 python scripts/graphbench.py > gpurun_out/il2/hl.jsonl 2> gpurun_out/il2/hl.err
rc=$?; echo "gb hl rc=$rc"; grep decode gpurun_out/il2/hl.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/il2/hl.err; exit $rc; }
exit 0
