#!/bin/bash
# round 4: new boundary tests on the GPU + the self-launched 2-rank rehearsal
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04a
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_codec_pipeline.py tests/test_gpu_lifecycle.py tests/test_gpu_compression.py > gpurun_out/r04a/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r04a/pytest.log
[ $rc -ne 0 ] && exit $rc
ZHIP_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --extra "" > gpurun_out/r04a/bench_rehearsal_2.json 2> gpurun_out/r04a/bench_rehearsal_2.err
rc=$?; echo "rehearsal rc=$rc"; cat gpurun_out/r04a/bench_rehearsal_2.json; tail -3 gpurun_out/r04a/bench_rehearsal_2.err
exit $rc
