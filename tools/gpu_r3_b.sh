#!/bin/bash
# GPU tests (RCCL world-1 + LDS kernels), bench with a forced one-rank RCCL group, LDS A/B.
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3b
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_kernels.py -k "rccl or lds or records_match" -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench_base.json 2> $OUT/bench_base.err || { tail -5 $OUT/bench_base.err; exit 1; }
echo "base   $(tail -1 $OUT/bench_base.json | cut -c100-180)"
TB_FORCE_PG=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench_pg.json 2> $OUT/bench_pg.err || { tail -5 $OUT/bench_pg.err; exit 1; }
echo "pg     $(tail -1 $OUT/bench_pg.json | cut -c100-180)"
TB_OUT=$OUT TB_WB_AB="10240 16384" bash tools/gpu_lds_quick.sh
