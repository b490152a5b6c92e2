#!/bin/bash
# round 3: k_decode_il skeleton arms: no table loads (512), no run end (4096), no publication (1073741824), CF lookups (131072)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03v
TUNES=0,512,4096,1073741824,131072,1073746432 COPIES=0 ROUNDS=7 timeout -k 10 300 python scripts/graphbench.py > gpurun_out/r03v/hl.jsonl 2> gpurun_out/r03v/hl.err
rc=$?; echo "gb headline rc=$rc"; grep -v scatterg gpurun_out/r03v/hl.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03v/hl.err; exit $rc; }
exit 0
