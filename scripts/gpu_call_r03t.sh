#!/bin/bash
# round 3: conflict-free-lookup timing arm (kTuneCfLookup) on k_decode_il, headline and C5
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03t
TUNES=0,131072,1 COPIES=0 ROUNDS=7 timeout -k 10 300 python scripts/graphbench.py > gpurun_out/r03t/hl.jsonl 2> gpurun_out/r03t/hl.err
rc=$?; echo "gb headline rc=$rc"; grep -v scatterg gpurun_out/r03t/hl.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03t/hl.err; exit $rc; }
exit 0
