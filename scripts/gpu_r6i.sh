#!/bin/bash
# Round 6: with groups of 32 workgroups in production, re-run the headline's
# round-5 arms whose effect depended on the access order: XCD-contiguous
# eighths (57) and no wave priority (56).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r6i}; mkdir -p "$O"
export TMPDIR=/tmp
OUT=$O ROUNDS=15 CONFIGS="headline" ARMS="prod=0:0,x8=0:57,np=0:56,prod2=0:0,x8b=0:57,npb=0:56" \
  bash scripts/gpu_arms.sh || exit $?
exit 0
