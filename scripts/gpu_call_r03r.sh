#!/bin/bash
# round 3: k_decode_lead (default sharding chain), il prologue arms, full bench
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03r
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03r/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03r/pytest.log; [ $rc -ne 0 ] && exit $rc
TUNES=0,16384,134217728 COPIES=0 ROUNDS=7 timeout -k 10 300 python scripts/graphbench.py > gpurun_out/r03r/hl.jsonl 2> gpurun_out/r03r/hl.err
rc=$?; echo "gb headline rc=$rc"; grep -v scatterg gpurun_out/r03r/hl.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03r/hl.err; exit $rc; }
timeout -k 10 600 python bench.py --steps 20 --warmup 10 > gpurun_out/r03r/bench.json 2> gpurun_out/r03r/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r03r/bench.json; tail -3 gpurun_out/r03r/bench.err
exit $rc
