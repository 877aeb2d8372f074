#!/bin/bash
# PMC counter passes over a short 1-GPU bench (one rocprofv3 run per counter group; counters are
# never combined with sys/runtime tracing). Output: gpurun_out/pmc/<pass>/...
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
OUT="$REPO/gpurun_out/pmc"
mkdir -p "$OUT"
STEPS=${TB_PROF_STEPS:-3}
# TB_PROF_ARGS: extra bench.py arguments (e.g. the config 5 long-document workload)
run_pass() {
  local name=$1; shift
  timeout -k 10 ${TB_PROF_TIMEOUT:-300} rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run \
    -- python3 "$REPO/bench.py" --steps $STEPS --warmup 1 $TB_PROF_ARGS > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
run_pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU &&
run_pass mem SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum &&
run_pass hbm FETCH_SIZE SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_FLAT SQ_INSTS_FLAT_LDS_ONLY &&
run_pass wr WRITE_SIZE SQ_INSTS_VMEM_WR
rc=$?
find "$OUT" -name "*counter_collection*.csv" | head
exit $rc
