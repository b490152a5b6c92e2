#!/bin/bash
# round 3: end-to-end leg alone, repeated, default (streaming-store packing)
# and memcpy packing, to see the box-to-box and run-to-run spread
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03ae
for i in 1 2; do
  for mode in nt memcpy; do
    if [ $mode = memcpy ]; then export ZARR_HIP_STAGE_COPY=memcpy; else unset ZARR_HIP_STAGE_COPY; fi
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --extra e2e --no-cpu-baseline > gpurun_out/r03ae/e2e_${mode}_$i.json 2> gpurun_out/r03ae/e2e_${mode}_$i.err
    rc=$?; echo "e2e $mode $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
    python -c "import json;e=json.load(open('gpurun_out/r03ae/e2e_${mode}_$i.json'))['extra']['e2e_c2_host'];print('$mode', e['host_to_host_GiBps'], e['host_to_hbm_decoded_GiBps'], e['pinned_store_to_hbm_decoded_GiBps'], e['local_store_to_hbm_decoded_GiBps'])"
  done
done
timeout -k 10 200 python scripts/host_bw.py > gpurun_out/r03ae/host_bw.jsonl 2> gpurun_out/r03ae/host_bw.err
rc=$?; echo "host_bw rc=$rc"; grep -E "raw pinned|H2D \+ D2H|threads=16 copy=nt" gpurun_out/r03ae/host_bw.jsonl
exit $rc
