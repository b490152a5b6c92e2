#!/bin/bash
# Round 6: the tuning tests (one process, the tuning build), the default bench,
# a rocprofv3 kernel-trace of the headline, and graph-timed A/B of the
# look-back arrival arms on the 128^3-chunk transposes.  Each GPU step under
# its own limit, stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r6c}; mkdir -p "$O"
export TMPDIR=/tmp
ZARR_HIP_ALLOW_LIB_OVERRIDE=1 ZHIP_LIB="$PWD/zarr-python_amd/zarr_hip/_lib/libzarrhip_tune.so" \
  timeout -k 10 600 python -u -m pytest tests -m "gpu and tuning" -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > "$O/pytest_tuning.log" 2>&1
rc=$?; echo "pytest tuning rc=$rc"; tail -3 "$O/pytest_tuning.log"; [ $rc -ne 0 ] && { tail -40 "$O/pytest_tuning.log"; exit $rc; }
timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; tail -c 400 "$O/bench.json"; [ $rc -ne 0 ] && { tail -20 "$O/bench.err"; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o hl -- python bench.py --steps 50 --extra "" \
  --no-cpu-baseline > "$O/bench_prof.json" 2> "$O/bench_prof.err"
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$O/bench_prof.err"; exit $rc; }
OUT=$O ROUNDS=15 CONFIGS="c3g" ARMS="prod=0:0,lb=0:62" bash scripts/gpu_arms.sh || exit $?
mkdir -p "$O/hl" && OUT=$O/hl ROUNDS=15 CONFIGS="headline" ARMS="prod=0:0,wt=0:64,bnt=0:65,prod2=0:0,wt2=0:64" \
  bash scripts/gpu_arms.sh || exit $?
ARMS="c3_128:0,c3_128:63,c3_128:0,c3_128:63" timeout -k 10 400 python scripts/encbench.py > "$O/enc_arms.jsonl" 2> "$O/enc_arms.err"
rc=$?; echo "enc rc=$rc"; cat "$O/enc_arms.jsonl"; [ $rc -ne 0 ] && { tail -5 "$O/enc_arms.err"; exit $rc; }
exit 0
