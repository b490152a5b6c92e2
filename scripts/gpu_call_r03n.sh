#!/bin/bash
# round 3, re-entry: baseline of the restored tree (tests, smoke, full bench, rocprof stats)
set -u
cd "$GRAFT_REPO_ROOT"
STEPS=20 PROFILE=1 bash scripts/gpu_round.sh
