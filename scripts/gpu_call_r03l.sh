set -u
cd "$GRAFT_REPO_ROOT"
ARMS="hl:0 hl:134217728 hl:1" PASSES="sq insts mem" bash scripts/gpu_arms_pmc.sh
