#!/bin/bash
# BASELINE config 5 (GopherRepetition 2..10-gram on ~50 KB documents): bench + per-phase cycle
# profile of the long-document kernels, plus the config 1 start-up check (1k rows, CLI path).
set -e
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT="$REPO/gpurun_out/c5"
mkdir -p "$OUT"
cd "$REPO"
C=$REPO/config/baseline
A="--config $C/gopher_rep_2_10.yaml --mean-bytes 51200 --docs-per-step ${TB_C5_DOCS:-4096} --pool 1024"
timeout -k 10 300 python bench.py $A --steps 10 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
tail -1 "$OUT/bench.json" | cut -c1-300
TB_PHASE_PROF=1 timeout -k 10 300 python bench.py $A --steps 3 --warmup 1 > "$OUT/phase_stdout.log" 2> "$OUT/phase_cycles.txt"
cat "$OUT/phase_cycles.txt" | tail -40
cd /tmp && export TMPDIR=/tmp
TB_SERIAL_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/serial" -o c5 \
  -- python3 "$REPO/bench.py" $A --steps 3 --warmup 1 > "$OUT/serial.log" 2>&1
K=$(find "$OUT/serial" -name "*kernel_trace.csv" | head -1)
python3 "$REPO/tools/prof_summary.py" "$K" > "$OUT/kernels_serialized.txt" 2>&1 || true
head -12 "$OUT/kernels_serialized.txt"
rm -f "$K"
cd "$REPO"
timeout -k 10 300 python tools/e2e_bench.py --docs 1000 --row-group 1000 --unit-rows 1000 --config $C/c4_only.yaml \
    --backend cpu --backend cuda --out /tmp/tb_c1 > "$OUT/c1_file.json" 2>&1
grep backend "$OUT/c1_file.json" | cut -c1-300
