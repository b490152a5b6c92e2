#!/bin/bash
# round 3: e2e legs alone, streaming-store vs memcpy packing (A/B), twice each; C5 host line alone
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03s
for i in 1 2; do
for m in nt memcpy; do
ZARR_HIP_STAGE_COPY=$m timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --extra e2e > gpurun_out/r03s/e2e_${m}_$i.json 2> gpurun_out/r03s/e2e_${m}_$i.err
rc=$?; echo "e2e $m $i rc=$rc"; python -c "import json,sys; d=json.loads(open('gpurun_out/r03s/e2e_${m}_$i.json').read().strip().splitlines()[-1]); print(d['extra']['e2e_c2_host'])"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03s/e2e_${m}_$i.err; exit $rc; }
done
done
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --extra c5 > gpurun_out/r03s/c5.json 2> gpurun_out/r03s/c5.err
rc=$?; echo "c5 rc=$rc"; python -c "import json,sys; d=json.loads(open('gpurun_out/r03s/c5.json').read().strip().splitlines()[-1]); print(d['extra']['c5_host_coalesced'])"
exit $rc
