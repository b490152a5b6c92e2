#!/bin/bash
# round 3 final-tree measurements: GPU tests, smoke, full bench, rocprof stats,
# torchrun N=1, 2-rank rehearsal on one GPU (gloo), PMC traffic passes
set -u
cd "$GRAFT_REPO_ROOT"
STEPS=20 PROFILE=1 TORCHRUN=1 REHEARSAL=1 REHEARSAL_EXTRA="c4,c5" PMC=1 bash scripts/gpu_round.sh
