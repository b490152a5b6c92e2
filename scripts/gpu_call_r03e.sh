set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gb
CONFIG=c4 TUNES=0,1,33554432 ROUNDS=5 timeout -k 10 600 python scripts/graphbench.py > gpurun_out/gb/c4.jsonl 2> gpurun_out/gb/c4.err
rc=$?; echo "gb c4 rc=$rc"; cat gpurun_out/gb/c4.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/gb/c4.err; exit $rc; }
CONFIG=headline TUNES=0,1,16777216,33554432 ROUNDS=5 timeout -k 10 600 python scripts/graphbench.py > gpurun_out/gb/hl.jsonl 2> gpurun_out/gb/hl.err
rc=$?; echo "gb hl rc=$rc"; cat gpurun_out/gb/hl.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/gb/hl.err; exit $rc; }
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --extra call > gpurun_out/gb/bench_call.json 2> gpurun_out/gb/bench_call.err
rc=$?; echo "bench call rc=$rc"; cat gpurun_out/gb/bench_call.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/gb/bench_call.err; exit $rc; }
exit 0
