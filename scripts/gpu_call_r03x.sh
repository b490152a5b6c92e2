#!/bin/bash
# round 3: final-library measurement (tests, smoke, bench, rocprof stats, PMC traffic)
set -u
cd "$GRAFT_REPO_ROOT"
STEPS=20 PROFILE=1 PMC=1 TORCHRUN=1 bash scripts/gpu_round.sh
