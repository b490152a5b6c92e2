#!/bin/bash
# Round 6: the byte-table chain arms (66 / 67) against production on another
# box, with the headline beside them (a box-speed reference).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r6e}; mkdir -p "$O"
export TMPDIR=/tmp
rocm-smi --showclocks > "$O/clocks_before.txt" 2>&1 || true
OUT=$O ROUNDS=15 CONFIGS="headline" ARMS="prod=0:0" bash scripts/gpu_arms.sh || exit $?
OUT=$O ROUNDS=15 CONFIGS="c3" ARMS="prod=0:0,bt=0:67,prod2=0:0,bt2=0:67" bash scripts/gpu_arms.sh || exit $?
OUT=$O ROUNDS=15 CONFIGS="c3g" ARMS="prod=0:0,bt=0:66,prod2=0:0,bt2=0:66" bash scripts/gpu_arms.sh || exit $?
rocm-smi --showclocks > "$O/clocks_after.txt" 2>&1 || true
exit 0
