#!/bin/bash
# Stage kernel cost per step type: serialized kernel time of one-step pipelines (config/ablate/),
# LDS kernel (TB_LDS_STAGE=1) vs generic. Output gpurun_out/ablate/.
cd "$(dirname "$0")/.."
OUT=gpurun_out/ablate
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
REPO=$GRAFT_REPO_ROOT
for cfg in gq gr_lines gr_top gr_dup fw; do
  for lds in 0 1; do
    TB_LDS_STAGE=$lds TB_SERIAL_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $REPO/$OUT/${cfg}_$lds -o t -- python3 $REPO/bench.py --config $REPO/config/ablate/$cfg.yaml --steps 3 --warmup 1 > $REPO/$OUT/${cfg}_$lds.log 2>&1 || { echo "fail $cfg $lds"; tail -3 $REPO/$OUT/${cfg}_$lds.log; exit 1; }
    tr=$(find $REPO/$OUT/${cfg}_$lds -name "*kernel_trace.csv" | head -1)
    python3 - "$tr" "$cfg" "$lds" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
t = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if "stage" in r["Kernel_Name"])
print("%-9s lds=%s stage kernels %.2f ms/step" % (sys.argv[2], sys.argv[3], t / 4 / 1e6))
PY
  done
done
