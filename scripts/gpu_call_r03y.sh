#!/bin/bash
# round 3: C4 publication-latency arm (kTuneNoTicket: no returning atomic),
# SQ counters of the current (XOR-swizzled) tile kernels, and the host-read
# fast path (MemoryStore batch values in one pass): staging tests, e2e phases
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03y
timeout -k 10 300 python -u -m pytest tests/test_gpu_staging.py tests/test_gpu_boundary.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03y/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03y/pytest.log; [ $rc -ne 0 ] && exit $rc
CONFIG=c4 TUNES=0,4,1,5 COPIES=0 ROUNDS=3 timeout -k 10 400 python scripts/graphbench.py > gpurun_out/r03y/c4.jsonl 2> gpurun_out/r03y/c4.err
rc=$?; echo "gb c4 rc=$rc"; grep -v scatterg_ gpurun_out/r03y/c4.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03y/c4.err; exit $rc; }
WINDOWS=4 CPROFILE=1 timeout -k 10 300 python scripts/e2e_profile.py > gpurun_out/r03y/e2e_profile.jsonl 2> gpurun_out/r03y/e2e_profile.err
rc=$?; echo "e2e profile rc=$rc"; cat gpurun_out/r03y/e2e_profile.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03y/e2e_profile.err; exit $rc; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --extra e2e --no-cpu-baseline > gpurun_out/r03y/bench_e2e.json 2> gpurun_out/r03y/bench_e2e.err
rc=$?; echo "bench e2e rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/r03y/bench_e2e.json'));print(json.dumps(d['extra']['e2e_c2_host']))"; [ $rc -ne 0 ] && exit $rc
TUNES=0 bash scripts/gpu_decpmc.sh > gpurun_out/r03y/decsq.log 2>&1
rc=$?; echo "decsq rc=$rc"; cat gpurun_out/r03y/decsq.log
exit $rc
