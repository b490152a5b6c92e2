set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/arms
for spec in "ARM=hl TUNE=0" "ARM=hl TUNE=1" "ARM=c4 TUNE=0" "ARM=c4 TUNE=1" "ARM=copy SIZE=4294967296 SPAN=4096 K=1 NT=1" "ARM=copy SIZE=4294967296 SPAN=32768 K=8 NT=1" "ARM=copy SIZE=67108864 SPAN=4096 K=1 NT=1"; do
  env $spec timeout -k 10 120 python scripts/arms.py >> gpurun_out/arms/timing.jsonl 2>> gpurun_out/arms/timing.err || { echo "arm failed: $spec"; tail -5 gpurun_out/arms/timing.err; exit 1; }
done
cat gpurun_out/arms/timing.jsonl
ARMS="hl:0 hl:1 c4:0 c4:1 copy:0:SIZE=4294967296,SPAN=4096,NT=1" PASSES="sq insts" bash scripts/gpu_arms_pmc.sh
