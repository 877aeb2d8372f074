#!/bin/bash
# ~1 MB documents (GopherRepetition 2-10-gram, 128 docs/step): serialized kernel stats and the
# stage workgroup's phase cycles.
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
REPO=$(pwd)
OUT=$REPO/gpurun_out/mbprof
mkdir -p $OUT
C=$REPO/config/baseline/gopher_rep_2_10.yaml
ARGS="--config $C --mean-bytes 1048576 --docs-per-step 128 --pool 32"
TB_PHASE_PROF=1 timeout -k 10 300 python bench.py $ARGS --steps 2 --warmup 1 > $OUT/phase.json 2> $OUT/phase.txt || { tail -5 $OUT/phase.txt; exit 1; }
grep -v amdgpu.ids $OUT/phase.txt | head -40
cd /tmp && export TMPDIR=/tmp
TB_SERIAL_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/serial -o t -- python3 $REPO/bench.py $ARGS --steps 3 --warmup 1 > $OUT/serial.log 2>&1 || { tail -5 $OUT/serial.log; exit 1; }
TR=$(find $OUT/serial -name "*kernel_trace.csv" | head -1)
python3 $REPO/tools/prof_summary.py "$TR" > $OUT/kernels_serialized.txt 2>&1
head -12 $OUT/kernels_serialized.txt
