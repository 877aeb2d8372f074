#!/bin/bash
# Serialized kernel time of the stage kernels: generic vs LDS hybrids (exclusive timings, no
# concurrency noise).
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/hyb2
mkdir -p $OUT
for cfg in "gen TB_LDS_STAGE=0" "h10k TB_LDS_STAGE=1 TB_LDS_GENERIC_ABOVE=10240" "h6k TB_LDS_STAGE=1 TB_LDS_GENERIC_ABOVE=6144" "lds TB_LDS_STAGE=1"; do
  set -- $cfg; name=$1; shift
  env "$@" bash tools/prof_current.sh > $OUT/prof_$name.log 2>&1 || { tail -5 $OUT/prof_$name.log; exit 1; }
  cp gpurun_out/cur/kernels_serialized.txt $OUT/k_$name.txt
  python3 - $OUT/k_$name.txt $name <<'PY'
import sys
tot = 0.0
for ln in open(sys.argv[1]):
    p = ln.split()
    if len(p) >= 5 and p[0].startswith("k_stage") and "blk" not in p[0]:
        tot += float(p[2])
print("%-6s stage wave kernels %.1f ms per 5 steps" % (sys.argv[2], tot))
PY
  grep "GPU busy per step" $OUT/k_$name.txt
done
