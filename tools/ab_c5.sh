#!/bin/bash
# Long-document kernel A/B on BASELINE config 5 (GopherRepetition 2..10-gram, ~50 KB documents):
# GPU tests, then the config 5 bench per kernel-library variant (tools/build_variant.sh NAME ...;
# VARIANTS="base name[:LDS_BYTES_BLK] ..."), then the main bench.
set -e
C=$GRAFT_REPO_ROOT/config/baseline
A="--config $C/gopher_rep_2_10.yaml --mean-bytes 51200 --docs-per-step 4096 --pool 1024 --steps 8 --warmup 2"
mkdir -p gpurun_out/c5ab
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; tail -1 gpurun_out/pytest_gpu.log
for VL in ${VARIANTS:-base}; do
  V=${VL%%:*}; LDS=${VL#*:}; [ "$LDS" = "$VL" ] && LDS=65536
  if [ $V = base ]; then L=""; else L="$GRAFT_REPO_ROOT/textblaster_amd/libtbhip_$V.so"; fi
  TB_LDS_BYTES_BLK=$LDS TB_HIP_LIB=$L timeout -k 10 200 python bench.py $A > gpurun_out/c5ab/$VL.json 2> gpurun_out/c5ab/$VL.err
  echo "$VL $(tail -1 gpurun_out/c5ab/$VL.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1; tail -1 gpurun_out/bench.log | cut -c1-200
