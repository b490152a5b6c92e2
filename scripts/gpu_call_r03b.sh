set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/land
for size in 4294967296 67108864; do
for sk in "4096 1" "8192 1" "8192 2" "16384 1" "16384 2" "16384 4" "32768 1" "32768 2" "32768 4" "32768 8" "65536 4" "65536 16"; do
  set -- $sk
  for nt in 3 1; do
    ARM=copy SIZE=$size SPAN=$1 K=$2 NT=$nt timeout -k 10 120 python scripts/arms.py >> gpurun_out/land/copy.jsonl 2>> gpurun_out/land/copy.err || { echo "arm failed $size $sk $nt"; tail -5 gpurun_out/land/copy.err; exit 1; }
  done
done
done
cat gpurun_out/land/copy.jsonl
