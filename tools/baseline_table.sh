#!/bin/bash
# Measures every BASELINE.json configuration that fits one MI355X (the 8-GPU scaling run is the
# driver's): GPU and CPU-path docs/s per config, JSON lines into gpurun_out/baseline/.
#   gpurun --timeout 1200 -- 'bash tools/baseline_table.sh'
# then: python tools/baseline_table.py gpurun_out/baseline   (prints the BASELINE.md table)
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/baseline
mkdir -p $O
T="timeout -k 10"
run() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  echo "== $name" >&2
  $T "$secs" "$@" > "$O/$name.json" 2> "$O/$name.err"
  local rc=$?
  tail -1 "$O/$name.json" >&2
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc" >&2; tail -20 "$O/$name.err" >&2; exit $rc; fi
}
C=config/baseline
# 1. C4QualityFilter only: 1k-row synthetic Parquet through the CLI path, and the in-memory step
run c1_file 300 python tools/e2e_bench.py --docs 1000 --row-group 1000 --unit-rows 1000 --config $C/c4_only.yaml \
    --backend cpu --backend cuda --out /tmp/tb_c1
run c1_cpu 300 python bench.py --config $C/c4_only.yaml --backend cpu --steps 5 --warmup 1
run c1_gpu 300 python bench.py --config $C/c4_only.yaml --steps 20 --warmup 5
# 2. C4 + GopherQuality + GopherRepetition, >= 10M ~1 KB docs (153 steps x the bench batch, 262,144 docs)
run c2_gpu 600 python bench.py --config $C/c4_gopher.yaml --steps 153 --warmup 5
run c2_cpu 300 python bench.py --config $C/c4_gopher.yaml --backend cpu --steps 3 --warmup 1
# 3. + LanguageDetectionFilter (bench.py default config)
run c3_gpu 300 python bench.py --steps 20 --warmup 5
run c3_cpu 300 python bench.py --backend cpu --steps 3 --warmup 1
# 5. GopherRepetition 2..10-gram on ~50 KB documents
run c5_gpu 600 python bench.py --config $C/gopher_rep_2_10.yaml --mean-bytes 51200 --docs-per-step 4096 --pool 1024 \
    --steps 20 --warmup 5
# 5b. the same filter on ~1 MB documents, 128 per step (the long-document path: pre-pass, split orders)
run c5mb_gpu 600 python bench.py --config $C/gopher_rep_2_10.yaml --mean-bytes 1048576 --docs-per-step 128 --pool 256 \
    --steps 20 --warmup 5
run c5_cpu 600 python bench.py --config $C/gopher_rep_2_10.yaml --mean-bytes 51200 --docs-per-step 4096 --pool 1024 \
    --backend cpu --steps 1 --warmup 1
# 4. (1-GPU point) CommonCrawl-shaped Parquet through the CLI path: read, decode, filter, write
run c4_file 900 python tools/e2e_bench.py --docs 20000000 --backend cuda --out /tmp/tb_c4
echo "baseline table done" >&2
