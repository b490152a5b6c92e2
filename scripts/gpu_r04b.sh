#!/bin/bash
# round 4: new boundary tests + 2-rank rehearsal (self-launched) + il publication arms
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04b
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_codec_pipeline.py tests/test_gpu_lifecycle.py tests/test_gpu_compression.py tests/test_gpu_cpp_example.py > gpurun_out/r04b/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r04b/pytest.log
[ $rc -ne 0 ] && [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --extra cpp > gpurun_out/r04b/bench_cpp.json 2> gpurun_out/r04b/bench_cpp.err
rc=$?; echo "bench cpp rc=$rc"; cat gpurun_out/r04b/bench_cpp.json; tail -3 gpurun_out/r04b/bench_cpp.err
exit $rc
ARMS="prod=0:0,tuned_nopub=1073741824:0,dv=0:1,prod2=0:0" timeout -k 10 300 python scripts/armbench.py > gpurun_out/r04b/arms_headline.jsonl 2> gpurun_out/r04b/arms_headline.err
rc=$?; echo "arms rc=$rc"; cat gpurun_out/r04b/arms_headline.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/r04b/arms_headline.err; exit $rc; }
ZHIP_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --extra "" > gpurun_out/r04b/bench_rehearsal_2.json 2> gpurun_out/r04b/bench_rehearsal_2.err
rc=$?; echo "rehearsal rc=$rc"; cat gpurun_out/r04b/bench_rehearsal_2.json; tail -3 gpurun_out/r04b/bench_rehearsal_2.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --extra cpp > gpurun_out/r04b/bench_cpp.json 2> gpurun_out/r04b/bench_cpp.err
rc=$?; echo "bench cpp rc=$rc"; cat gpurun_out/r04b/bench_cpp.json; tail -3 gpurun_out/r04b/bench_cpp.err
exit $rc
