#!/bin/bash
# Counter passes (each its own rocprofv3 run, --pmc only) over one-arm
# processes (scripts/arms.py).  ARMS = space-separated "ARM:TUNE[:k=v,...]"
# specs; PASSES = names of the counter groups below.  Counters the box's
# rocprofv3 does not list are dropped from a group before the run.
# Output: gpurun_out/arms/<arm>.<pass>.summary.json per arm and pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"; O="$R/gpurun_out/arms"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
if [ ! -s "$O/counters.txt" ]; then
  timeout -s KILL 60 rocprofv3 -L > "$O/counters.txt" 2>&1 || true
fi
declare -A GRP
GRP[sq]="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
GRP[insts]="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_BRANCH"
GRP[mem]="TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TD_BUSY_avr GRBM_GUI_ACTIVE"
GRP[mem2]="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TA_TA_BUSY_sum TD_TD_BUSY_sum"
GRP[fetch]="FETCH_SIZE"
GRP[write]="WRITE_SIZE"
listed() {  # keep the counters rocprofv3 -L names
  local out=""
  for c in $1; do
    base="${c%_sum}"; base="${base%_avr}"
    if grep -q -w -e "$c" -e "$base" "$O/counters.txt"; then out="$out $c"; else echo "drop $c" >&2; fi
  done
  echo $out
}
for spec in ${ARMS:-hl:0}; do
  IFS=: read -r arm tune kv <<< "$spec"
  envs="ARM=$arm TUNE=${tune:-0}"
  [ -n "${kv:-}" ] && envs="$envs ${kv//,/ }"
  name="${arm}_t${tune:-0}${kv:+_${kv//[,=]/_}}"
  for pass in ${PASSES:-sq}; do
    ctrs=$(listed "${GRP[$pass]}")
    [ -z "$ctrs" ] && { echo "$name $pass: no counters"; continue; }
    d="$O/$name.$pass"
    env $envs timeout -s KILL 150 rocprofv3 --pmc $ctrs -d "$d" -o pmc --output-format csv -- python "$R/scripts/arms.py" > "$d.json" 2> "$d.err"
    rc=$?; echo "$name $pass rc=$rc $(cat "$d.json" 2>/dev/null)"
    if [ $rc -ne 0 ]; then tail -5 "$d.err"; exit $rc; fi
    needle=k_decode; [ "$arm" = copy ] && needle=k_copy
    python "$R/scripts/pmc_summary.py" "$d" "$needle" "$d.summary.json" > /dev/null
    python -c "import json;d=json.load(open('$d.summary.json'));print('  ', {k:round(v) for k,v in d['median_per_launch_KiB'].items()})"
  done
done
