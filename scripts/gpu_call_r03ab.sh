#!/bin/bash
# round 3: lean-prologue k_decode_il address mispredictions (diagnostic counter)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03ab
timeout -k 10 200 python scripts/il_lean_miss.py > gpurun_out/r03ab/miss.jsonl 2> gpurun_out/r03ab/miss.err
rc=$?; echo "miss rc=$rc"; cat gpurun_out/r03ab/miss.jsonl; [ $rc -ne 0 ] && tail -5 gpurun_out/r03ab/miss.err
exit $rc
