#!/bin/bash
# Long documents: BASELINE config 5 (~50 KB docs, GopherRepetition 2-10-gram) and
# ~1 MB documents at 128 and 384 docs per step; then the knob sweep of the headline config.
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/long
mkdir -p $OUT
C=config/baseline/gopher_rep_2_10.yaml
one() { local name=$1; shift; env timeout -k 10 300 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print('%-12s %.1f docs/s %.3f ms/step %.2f GB/s' % ('$name', d['value'], d['ms_per_step'], d['bytes_per_sec']/1e9))"; }
one c5 --config $C --mean-bytes 51200 --docs-per-step 4096 --pool 1024 --steps 10 --warmup 2
one mb128 --config $C --mean-bytes 1048576 --docs-per-step 128 --pool 32 --steps 5 --warmup 1
one mb384 --config $C --mean-bytes 1048576 --docs-per-step 384 --pool 32 --steps 5 --warmup 1
TB_HUGE_DOC_BYTES=0 one mb128_512 --config $C --mean-bytes 1048576 --docs-per-step 128 --pool 32 --steps 5 --warmup 1
TB_HUGE_DOC_BYTES=0 one mb384_512 --config $C --mean-bytes 1048576 --docs-per-step 384 --pool 32 --steps 5 --warmup 1
