#!/bin/bash
# One GPU-box session of timing arms (measurement only), every step under its
# own time limit, stopping at the first failure:
#   TESTS     optional pytest -k expression over tests/ -m gpu, run first
#   CONFIGS   scripts/armbench.py configs (headline share8 share4 c3 c3g c4),
#             each with ARMS = "name=ablation_bits:ZHIP_TUNE_ARM,..."
#   ENC_ARMS  scripts/encbench.py arms ("c2:0,c2:1,c3_64:0,...")
#   STAMPS    optional WORLD values for scripts/stamps.py (tuning build; "1 8"),
#             for each kernel arm of STAMP_ARMS (default "0")
#   PROF      "1": scripts/prof_uncached.py (SEL full / bench) and
#             scripts/prof_c5host.py
#   OUT       output directory under gpurun_out/ (default gpurun_out/arms_run)
# e.g. the round-4 publication arms:
#   OUT=gpurun_out/pub CONFIGS="headline share8 c3" ARMS="prod=0:0,ret16=0:1,dv=0:2" \
#     gpurun --timeout 900 -- 'bash scripts/gpu_arms.sh'
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/arms_run}; mkdir -p "$O"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "$TESTS" > "$O/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -1 "$O/pytest.log"
  [ $rc -ne 0 ] && exit $rc
fi
for a in ${STAMP_ARMS:-0}; do for w in ${STAMPS:-}; do  # per-workgroup phase stamps (WORLD=w: rank 0's share; ARM=a)
  WORLD=$w TUNE=${STAMP_TUNE:-0} ARM=$a STAMPS_OUT="$O/stamps_w${w}_a$a.npz" timeout -k 10 300 python scripts/stamps.py \
    > "$O/stamps_w${w}_a$a.jsonl" 2> "$O/stamps_w${w}_a$a.err"
  rc=$?; echo "stamps w=$w arm=$a rc=$rc"; cat "$O/stamps_w${w}_a$a.jsonl"
  [ $rc -ne 0 ] && { tail -5 "$O/stamps_w${w}_a$a.err"; exit $rc; }
done; done
for cfg in ${CONFIGS:-}; do
  CONFIG=$cfg ARMS="${ARMS:-prod=0:0}" timeout -k 10 300 python scripts/armbench.py > "$O/arms_$cfg.jsonl" 2> "$O/arms_$cfg.err"
  rc=$?; echo "arms $cfg rc=$rc"; cat "$O/arms_$cfg.jsonl"
  [ $rc -ne 0 ] && { tail -5 "$O/arms_$cfg.err"; exit $rc; }
done
if [ -n "${ENC_ARMS:-}" ]; then
  ARMS="$ENC_ARMS" timeout -k 10 500 python scripts/encbench.py > "$O/enc_arms.jsonl" 2> "$O/enc_arms.err"
  rc=$?; echo "enc rc=$rc"; cat "$O/enc_arms.jsonl"
  [ $rc -ne 0 ] && { tail -5 "$O/enc_arms.err"; exit $rc; }
fi
if [ "${PROF:-0}" = "1" ]; then
  for s in full bench; do
    SEL=$s timeout -k 10 200 python scripts/prof_uncached.py > "$O/prof_uncached_$s.jsonl" 2> "$O/prof_uncached_$s.err"
    rc=$?; echo "prof_uncached $s rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
  timeout -k 10 500 python scripts/prof_c5host.py > "$O/prof_c5host.jsonl" 2> "$O/prof_c5host.err"
  rc=$?; echo "prof_c5host rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
exit 0
