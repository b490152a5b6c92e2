#!/bin/bash
# round 3: k_decode_il arms -- lane multiply in registers (kTuneIlRegMul, 32)
# and the same with 24 KiB of LDS at 6 workgroups per CU (kTuneIlOcc6,
# 4194304): bench runs (output and CRC statuses checked) then graph-timed
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03aa
for tune in 32 4194304; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extra "" --no-cpu-baseline --tune $tune > gpurun_out/r03aa/bench_t$tune.json 2> gpurun_out/r03aa/bench_t$tune.err
  rc=$?; echo "bench tune=$tune rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03aa/bench_t$tune.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/r03aa/bench_t$tune.json'));r=d['roofline'];print(d['value'], r['kernel_ms_avg'], r['frac'])"
done
TUNES=0,32,4194304,0,32,4194304 COPIES=0 ROUNDS=5 timeout -k 10 300 python scripts/graphbench.py > gpurun_out/r03aa/hl.jsonl 2> gpurun_out/r03aa/hl.err
rc=$?; echo "gb headline rc=$rc"; grep -v "scatter" gpurun_out/r03aa/hl.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03aa/hl.err; exit $rc; }
for n in 8; do
  for tune in 0 32 4194304; do
    WORLD_SIZE=$n RANK=0 timeout -k 10 200 python bench.py --steps 50 --warmup 10 --extra "" --no-cpu-baseline --tune $tune > gpurun_out/r03aa/n${n}_t${tune}.json 2> gpurun_out/r03aa/n${n}_t${tune}.err
    rc=$?; echo "n=$n tune=$tune rc=$rc"; [ $rc -ne 0 ] && exit $rc
    python -c "import json;d=json.load(open('gpurun_out/r03aa/n${n}_t${tune}.json'));r=d['roofline'];print(d['value'], r['kernel_ms_avg'])"
  done
done
