#!/bin/bash
# One GPU-box session: tests, smoke, short bench, rocprof kernel stats.
# Stops at the first crash/timeout (exit codes other than 0/1 from pytest).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-50}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest_gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 10 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps "$STEPS" --warmup 10 --no-cpu-baseline --extra "" > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/bench_prof.err"
  rc=$?; echo "rocprof rc=$rc"
  find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name "*stats*" | head
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ "${TORCHRUN:-0}" = "1" ]; then
  cd "$GRAFT_REPO_ROOT"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --extra "" > gpurun_out/bench_torchrun.json 2> gpurun_out/bench_torchrun.err
  rc=$?; echo "torchrun bench rc=$rc"; cat gpurun_out/bench_torchrun.json
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_torchrun.err; exit $rc; fi
fi
if [ "${REHEARSAL:-0}" = "1" ]; then
  # the N>1 code path with 2 ranks on this one GPU (gloo group; not a scaling number)
  cd "$GRAFT_REPO_ROOT"
  ZHIP_BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 20 --warmup 5 --extra "${REHEARSAL_EXTRA:-c4,c5}" > gpurun_out/bench_rehearsal2.json 2> gpurun_out/bench_rehearsal2.err
  rc=$?; echo "rehearsal bench rc=$rc"; cat gpurun_out/bench_rehearsal2.json
  if [ $rc -ne 0 ]; then tail -15 gpurun_out/bench_rehearsal2.err; exit $rc; fi
fi
if [ "${PMC:-0}" = "1" ]; then
  bash "$GRAFT_REPO_ROOT/scripts/gpu_pmc.sh"
  rc=$?
fi
exit $rc
