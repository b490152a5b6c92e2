#!/bin/bash
# round 3: tests (incl. default-sharding-chain fusion), full bench, rocprof, e2e phase profile
set -u
cd "$GRAFT_REPO_ROOT"
STEPS=20 PROFILE=1 bash scripts/gpu_round.sh || exit $?
mkdir -p gpurun_out/e2e
CPROFILE=1 WINDOWS=4 timeout -k 10 300 python scripts/e2e_profile.py > gpurun_out/e2e/memory.jsonl 2> gpurun_out/e2e/memory.err
rc=$?; echo "e2e memory rc=$rc"; cat gpurun_out/e2e/memory.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/e2e/memory.err; exit $rc; }
STORE=pinned WINDOWS=4 timeout -k 10 300 python scripts/e2e_profile.py > gpurun_out/e2e/pinned.jsonl 2> gpurun_out/e2e/pinned.err
rc=$?; echo "e2e pinned rc=$rc"; cat gpurun_out/e2e/pinned.jsonl
exit $rc
