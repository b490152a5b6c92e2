#!/bin/bash
# round 3: lean pair prologue (one kernarg batch) vs k_decode_il; host bandwidth landscape
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03p
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03p/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03p/pytest.log; [ $rc -ne 0 ] && exit $rc
TUNES=0,134217728,134217729 COPIES=0 ROUNDS=5 timeout -k 10 300 python scripts/graphbench.py > gpurun_out/r03p/hl.jsonl 2> gpurun_out/r03p/hl.err
rc=$?; echo "gb headline rc=$rc"; cat gpurun_out/r03p/hl.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03p/hl.err; exit $rc; }
CONFIG=c4 TUNES=0,134217728 COPIES=0 ROUNDS=3 timeout -k 10 300 python scripts/graphbench.py > gpurun_out/r03p/c4.jsonl 2> gpurun_out/r03p/c4.err
rc=$?; echo "gb c4 rc=$rc"; grep -v scatterg_ gpurun_out/r03p/c4.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03p/c4.err; exit $rc; }
timeout -k 10 300 python scripts/host_bw.py > gpurun_out/r03p/host_bw.jsonl 2> gpurun_out/r03p/host_bw.err
rc=$?; echo "host_bw rc=$rc"; cat gpurun_out/r03p/host_bw.jsonl
exit $rc
