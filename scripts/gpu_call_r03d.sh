set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/land
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest_gpu rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
: > gpurun_out/land/copy2.jsonl
for size in 4294967296 67108864; do
  for spec in "MODE=wave K=8" "MODE=wave K=16" "MODE=wave K=4" "MODE=il K=8 SPAN=8" "MODE=il K=16 SPAN=8" "MODE=il K=8 SPAN=4" "MODE=span SPAN=32768 K=8" "MODE=span SPAN=4096 K=1"; do
    env ARM=copy SIZE=$size NT=3 $spec timeout -k 10 120 python scripts/arms.py >> gpurun_out/land/copy2.jsonl 2>> gpurun_out/land/copy2.err || { echo "arm failed $size $spec"; tail -5 gpurun_out/land/copy2.err; exit 1; }
  done
done
cat gpurun_out/land/copy2.jsonl
: > gpurun_out/land/pair.jsonl
for arm in hl c4; do
  for tune in 0 16777216 33554432 50331648 64; do
    ARM=$arm TUNE=$tune timeout -k 10 120 python scripts/arms.py >> gpurun_out/land/pair.jsonl 2>> gpurun_out/land/pair.err || { echo "arm failed $arm $tune"; tail -5 gpurun_out/land/pair.err; exit 1; }
  done
done
cat gpurun_out/land/pair.jsonl
