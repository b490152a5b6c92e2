#!/bin/bash
# round 3: rank 0's share of the strong-scaled headline (see r03z) with the
# lean predicted prologue (kTuneIlLean) vs production, and a rocprof kernel
# summary of rank 0 at N = 8 (kernel duration vs graph span per step)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03z2
for n in 1 2 4 8; do
  for tune in 0 16384; do
    WORLD_SIZE=$n RANK=0 timeout -k 10 200 python bench.py --steps 50 --warmup 10 --extra "" --no-cpu-baseline --tune $tune > gpurun_out/r03z2/n${n}_t${tune}.json 2> gpurun_out/r03z2/n${n}_t${tune}.err
    rc=$?; echo "n=$n tune=$tune rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03z2/n${n}_t${tune}.err; exit $rc; }
    python -c "import json;d=json.load(open('gpurun_out/r03z2/n${n}_t${tune}.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms_avg'], r['frac'])"
  done
done
cd /tmp && export TMPDIR=/tmp
WORLD_SIZE=8 RANK=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r03z2/prof8" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 10 --no-cpu-baseline --extra "" > "$GRAFT_REPO_ROOT/gpurun_out/r03z2/prof8.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r03z2/prof8.err"
rc=$?; echo "rocprof n8 rc=$rc"; grep -h k_decode "$GRAFT_REPO_ROOT"/gpurun_out/r03z2/prof8/*kernel_stats.csv | cut -c1-200
exit $rc
