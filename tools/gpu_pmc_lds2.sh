#!/bin/bash
# PMC passes on the LDS stage kernels (single-wave variants: TB_LDS_WAVE_BYTES=0) for the bench
# pipeline and the FineWeb-only ablation. Output gpurun_out/pmc2/.
cd "$(dirname "$0")/.."
REPO=$(pwd)
OUT=$REPO/gpurun_out/pmc2
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TB_LDS_STAGE=1 TB_LDS_WAVE_BYTES=0
cd /tmp && export TMPDIR=/tmp
run_pass() {
  local name=$1 cfg=$2; shift 2
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run \
    -- python3 "$REPO/bench.py" --config $REPO/$cfg --steps 2 --warmup 1 > "$OUT/$name.log" 2>&1
  local rc=$?; echo "pass $name rc=$rc"; return $rc
}
for c in fw bench; do
  cfg=config/ablate/fw.yaml; [ $c = bench ] && cfg=config/bench_pipeline.yaml
  run_pass ${c}_a $cfg SQ_WAVES SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES &&
  run_pass ${c}_b $cfg SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INST_CYCLES_SALU &&
  run_pass ${c}_c $cfg SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VSKIPPED SQ_LEVEL_WAVES SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU SQ_CYCLES || exit 1
  python3 $REPO/tools/pmc_summary.py $(find $OUT -path "*${c}_*" -name "*counter_collection*.csv") > $OUT/${c}_summary.txt 2>&1
done
grep -A 30 "k_stage_lds" $OUT/fw_summary.txt | head -70
