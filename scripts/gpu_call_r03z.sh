#!/bin/bash
# round 3: rank 0's share of the strong-scaled headline at N = 2, 4, 8, timed
# alone on one GPU (WORLD_SIZE / RANK without a process group: no barrier,
# rank 0's step time only -- an estimate of the driver's N-GPU numbers, not a
# scaling measurement), production kernel and the pair kernel (kTuneNoIl)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03z
for n in 2 4 8; do
  for tune in 0 134217728; do
    WORLD_SIZE=$n RANK=0 timeout -k 10 200 python bench.py --steps 50 --warmup 10 --extra "" --no-cpu-baseline --tune $tune > gpurun_out/r03z/n${n}_t${tune}.json 2> gpurun_out/r03z/n${n}_t${tune}.err
    rc=$?; echo "n=$n tune=$tune rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03z/n${n}_t${tune}.err; exit $rc; }
    python -c "import json;d=json.load(open('gpurun_out/r03z/n${n}_t${tune}.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms_avg'], r['frac'])"
  done
done
