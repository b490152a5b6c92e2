#!/bin/bash
# round 3: per-workgroup phase stamps of k_decode_pair (kTuneStamp) for rank
# 0's share of the strong-scaled headline at N = 8 and N = 1: where a lone
# workgroup's ~9 us goes when each CU holds one
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03z3
for w in 8 1; do
  WORLD=$w TUNE=134217728 timeout -k 10 200 python scripts/stamps.py > gpurun_out/r03z3/stamps_w$w.jsonl 2> gpurun_out/r03z3/stamps_w$w.err
  rc=$?; echo "stamps world=$w rc=$rc"; cat gpurun_out/r03z3/stamps_w$w.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03z3/stamps_w$w.err; exit $rc; }
done
exit 0
