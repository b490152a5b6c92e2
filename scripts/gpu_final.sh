#!/bin/bash
# Round 6 final evidence run on the shipped library (measurement only):
#   1. PMC passes of the headline (FETCH_SIZE, WRITE_SIZE: separate runs)
#      -> $O/pmc_traffic.json, copied to profiles/r06/pmc_traffic.json so the
#      bench below reports `traffic` for this library;
#   2. the default bench.py line -> $O/bench.json;
#   3. rocprofv3 --kernel-trace --stats of the headline and of each group of
#      config lines (bench.py --extra-only --extra X) -> $O/prof/<run>/;
#   4. scripts/rocprof_table.py -> $O/frac_table.json.
# Every GPU step under its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
O=${OUT:-gpurun_out/final}; mkdir -p "$O/prof" "$O/pmc"
export TMPDIR=/tmp
if [ "${SKIP_PMC:-0}" != "1" ]; then
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $grp -d "$R/$O/pmc/p$i" -o pmc --output-format csv -- \
      python "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --extra "" > "$R/$O/pmc/p$i.json" \
      2> "$R/$O/pmc/p$i.err")
    rc=$?; echo "pmc $grp rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$O/pmc/p$i.err"; exit $rc; }
  done
  python scripts/pmc_summary.py "$O/pmc" k_decode "$O/pmc_traffic.json" || exit $?
  mkdir -p profiles/r06 && cp "$O/pmc_traffic.json" profiles/r06/pmc_traffic.json
fi
timeout -k 10 700 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; tail -c 300 "$O/bench.json"; echo; [ $rc -ne 0 ] && { tail -20 "$O/bench.err"; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof/hl" -o hl -- python bench.py --steps 50 --extra "" \
  --no-cpu-baseline > "$O/prof/hl.json" 2> "$O/prof/hl.err"
rc=$?; echo "rocprof hl rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$O/prof/hl.err"; exit $rc; }
for x in ${RUNS:-c1 c2 c3 c4 c5 enc cpp}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof/$x" -o $x -- python bench.py --extra-only \
    --extra $x --steps 20 --no-host-legs > "$O/prof/$x.json" 2> "$O/prof/$x.err"
  rc=$?; echo "rocprof $x rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$O/prof/$x.err"; exit $rc; }
done
python scripts/rocprof_table.py "$O/bench.json" "$O/prof" "$O/frac_table.json" || exit $?
exit 0
