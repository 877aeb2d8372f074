#!/bin/bash
# HBM write bytes per kernel for two kernel libraries (default build vs TB_HIP_LIB=$1):
# one rocprofv3 --pmc pass each (WRITE_SIZE: 2 of the 4 TCC counters one run holds), 3 timed bench steps.
#   bash tools/pmc_write_ab.sh /root/repo/textblaster_amd/libtbhip_X.so  -> gpurun_out/${OUT:-pmcw}/
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
D="$REPO/gpurun_out/${OUT:-pmcw}"
mkdir -p "$D"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in default variant; do
  if [ $v = variant ]; then export TB_HIP_LIB=$1; fi
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_VMEM_WR SQ_INSTS_FLAT \
    --output-format csv -d "$D/$v" -o run -- python3 "$REPO/bench.py" --steps 3 --warmup 1) > "$D/$v.log" 2>&1 || exit 1
  python3 "$REPO/tools/pmc_summary.py" $(find "$D/$v" -name '*counter_collection.csv') --docs 1048576 > "$D/$v.txt" 2>&1
  find "$D/$v" -name '*.csv' -size +20M -delete
done
