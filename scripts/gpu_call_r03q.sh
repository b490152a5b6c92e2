#!/bin/bash
# round 3: lean + predicted k_decode_il prologue (vs kTuneIlOld, vs pair), e2e with streaming-store packing
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03q
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03q/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03q/pytest.log; [ $rc -ne 0 ] && exit $rc
TUNES=0,16384,134217728,1 COPIES=0 ROUNDS=7 timeout -k 10 300 python scripts/graphbench.py > gpurun_out/r03q/hl.jsonl 2> gpurun_out/r03q/hl.err
rc=$?; echo "gb headline rc=$rc"; grep -v scatterg gpurun_out/r03q/hl.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03q/hl.err; exit $rc; }
WINDOWS=4 timeout -k 10 300 python scripts/e2e_profile.py > gpurun_out/r03q/e2e_memory.jsonl 2> gpurun_out/r03q/e2e_memory.err
rc=$?; echo "e2e memory rc=$rc"; cat gpurun_out/r03q/e2e_memory.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03q/e2e_memory.err; exit $rc; }
STORE=pinned WINDOWS=4 timeout -k 10 300 python scripts/e2e_profile.py > gpurun_out/r03q/e2e_pinned.jsonl 2> gpurun_out/r03q/e2e_pinned.err
rc=$?; echo "e2e pinned rc=$rc"; cat gpurun_out/r03q/e2e_pinned.jsonl
exit $rc
