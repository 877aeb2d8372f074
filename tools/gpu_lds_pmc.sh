#!/bin/bash
# Phase cycles + PMC passes of the LDS stage kernel (gpurun_out/ldspmc/).
cd "$(dirname "$0")/.."
REPO=$(pwd)
OUT=$REPO/gpurun_out/ldspmc
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
TB_PHASE_PROF=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $OUT/phase_stdout.log 2> $OUT/phase_cycles.txt || { tail -5 $OUT/phase_cycles.txt; exit 1; }
head -40 $OUT/phase_cycles.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_avail.txt 2>&1 || true
run_pass() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run \
    -- python3 "$REPO/bench.py" --steps 2 --warmup 1 > "$OUT/$name.log" 2>&1
  local rc=$?; echo "pass $name rc=$rc"; return $rc
}
run_pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU &&
run_pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS
rc=$?
python3 $REPO/tools/pmc_summary.py $(find $OUT -name "*counter_collection*.csv") > $OUT/pmc_per_kernel.txt 2>&1
head -60 $OUT/pmc_per_kernel.txt
exit $rc
