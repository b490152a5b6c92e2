set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/il
# correctness first: the whole GPU suite with k_decode_il forced wherever a layout admits it
ZHIP_TUNE=67108864 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/il/pytest_il.log 2>&1
rc=$?
echo "pytest (il forced) rc=$rc"; tail -15 gpurun_out/il/pytest_il.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/il/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/il/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
CONFIG=c4 TUNES=0,134217728,1 ROUNDS=5 timeout -k 10 600 python scripts/graphbench.py > gpurun_out/il/c4.jsonl 2> gpurun_out/il/c4.err
rc=$?; echo "gb c4 rc=$rc"; cat gpurun_out/il/c4.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/il/c4.err; exit $rc; }
CONFIG=headline TUNES=0,67108864 ROUNDS=5 timeout -k 10 600 python scripts/graphbench.py > gpurun_out/il/hl.jsonl 2> gpurun_out/il/hl.err
rc=$?; echo "gb hl rc=$rc"; cat gpurun_out/il/hl.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/il/hl.err; exit $rc; }
exit 0
