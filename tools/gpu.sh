#!/bin/bash
# The one GPU-box driver (run through gpurun): every step has its own time limit, steps are
# chained so that a failure or timeout stops everything after it, outputs go to gpurun_out/$OUT.
#
#   bash tools/gpu.sh <step> [<step> ...]          e.g.  gpurun -- 'bash tools/gpu.sh test bench prof'
#
# steps:
#   test        pytest -m gpu (one process) + __graft_entry__.smoke()          -> pytest.log, smoke.log
#   tests=K     pytest -m gpu -k K (a subset)                                    -> pytest.log
#   bench       bench.py --steps $STEPS --warmup $WARMUP $BENCH_ARGS (the driver's 20 / 5)  -> bench.json
#   prof        serialized-stream kernel trace (exclusive kernel times, tools/prof_summary.py)
#               + TB_TUNE=phase_prof=1 per-phase wave cycles                         -> kernels_serialized.txt, phase_cycles.txt
#   pmc         PMC counter passes (one rocprofv3 run per counter group, no tracing) -> pmc_per_kernel.txt
#   ab          interleaved A/B of env settings: AB="TB_TUNE=slots=2,streams=6;TB_HIP_LIB=x.so TB_TUNE=slots=3"
#               (space-separated settings, ';'-separated env assignments), REPS repetitions,
#               serialized kernel stats + bench each
#   timeline    kernel + memory-copy trace of a few steps (tools/prof_summary.py per-step timeline)
#   e2e         Parquet -> Parquet end to end (tools/e2e_bench.py $E2E_ARGS)   -> e2e.json
# env: OUT (default r), STEPS (bench steps, 20), WARMUP (5), BENCH_ARGS (extra bench.py args, also used by
#      prof / pmc / ab / timeline), AB, REPS (1).
set -o pipefail
REPO=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$REPO" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
D="$REPO/gpurun_out/${OUT:-r}"
mkdir -p "$D"
STEPS=${STEPS:-20}
WARMUP=${WARMUP:-5}

kstats() {  # kstats <dir> <log> [env...]: serialized kernel trace of a short bench
  local dir=$1 log=$2 a tune="" envs=(); shift 2
  for a in "$@"; do  # one stream for everything (exclusive kernel times) on top of the setting's TB_TUNE
    if [[ $a == TB_TUNE=* ]]; then tune=${a#TB_TUNE=}; else envs+=("$a"); fi
  done
  (cd /tmp && export TMPDIR=/tmp && env "${envs[@]}" TB_TUNE="streams=serial${tune:+,$tune}" timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d "$dir" -o k -- python3 "$REPO/bench.py" --steps 4 --warmup 1 $BENCH_ARGS) > "$log" 2>&1
}

step_test() {
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$D/pytest.log" 2>&1
  local rc=$?
  tail -5 "$D/pytest.log"
  [ $rc -eq 0 ] || return $rc
  timeout -k 10 300 python __graft_entry__.py smoke > "$D/smoke.log" 2>&1
  rc=$?
  tail -3 "$D/smoke.log"
  return $rc
}

step_tests() {
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "$1" > "$D/pytest.log" 2>&1
  local rc=$?
  tail -5 "$D/pytest.log"
  return $rc
}

step_bench() {
  timeout -k 10 400 python3 bench.py --steps $STEPS --warmup $WARMUP $BENCH_ARGS > "$D/bench.json" 2> "$D/bench.err"
  local rc=$?
  cat "$D/bench.json"
  return $rc
}

step_prof() {
  kstats "$D/serial" "$D/serial.log" || { tail -5 "$D/serial.log"; return 1; }
  python3 tools/prof_summary.py "$(find "$D/serial" -name '*kernel_trace.csv' | head -1)" > "$D/kernels_serialized.txt" 2>&1
  find "$D/serial" -name '*kernel_trace.csv' -delete
  head -14 "$D/kernels_serialized.txt"
  TB_TUNE=phase_prof=1 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 $BENCH_ARGS > "$D/phase_bench.json" \
    2> "$D/phase_cycles.txt" || { tail -5 "$D/phase_cycles.txt"; return 1; }
  grep -v amdgpu.ids "$D/phase_cycles.txt" | head -30
}

pmc_pass() {  # pmc_pass <name> <counters...>
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc "$@" --output-format csv -d "$D/pmc/$name" \
    -o run -- python3 "$REPO/bench.py" --steps 3 --warmup 1 $BENCH_ARGS) > "$D/pmc/$name.log" 2>&1
}

step_pmc() {
  mkdir -p "$D/pmc"
  pmc_pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
    SQ_INSTS_SALU &&
  pmc_pass mem SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum &&
  pmc_pass hbm FETCH_SIZE SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_FLAT SQ_INSTS_FLAT_LDS_ONLY &&
  pmc_pass wr WRITE_SIZE SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES || return 1
  # documents per PMC run: (3 timed + 1 warmup steps) x bench.py's 262,144 per step unless
  # BENCH_ARGS changes the batch (then set PMC_DOCS), so the summary prints bytes per document
  python3 tools/pmc_summary.py $(find "$D/pmc" -name '*counter_collection.csv') --docs ${PMC_DOCS:-1048576} \
    > "$D/pmc_per_kernel.txt" 2>&1
  find "$D/pmc" -name '*.csv' -size +20M -delete
  head -40 "$D/pmc_per_kernel.txt"
}

step_ab() {
  local rep i=0
  for rep in $(seq 1 ${REPS:-1}); do
    i=0
    for S in $AB; do
      i=$((i + 1))
      local E
      E=$(echo "$S" | tr ';' ' ')
      kstats "$D/ab_r${rep}_$i" "$D/ab_r${rep}_$i.log" $E || { tail -5 "$D/ab_r${rep}_$i.log"; return 1; }
      local T
      T=$(find "$D/ab_r${rep}_$i" -name '*kernel_trace.csv' | head -1)
      {
        echo "== rep $rep: $S"
        python3 tools/prof_summary.py "$T" 2>&1 | sed -n 2,9p
        python3 tools/prof_summary.py "$T" 2>&1 | grep "GPU busy per step"
        env $E timeout -k 10 300 python3 bench.py --steps $STEPS --warmup $WARMUP $BENCH_ARGS 2>/dev/null | cut -c1-160
      } >> "$D/ab.txt"
      rm -f "$T"
    done
  done
  cat "$D/ab.txt"
}

step_timeline() {
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d "$D/tl" -o t -- python3 "$REPO/bench.py" --steps 5 --warmup 2 $BENCH_ARGS) > "$D/timeline.log" 2>&1 || return 1
  python3 tools/prof_summary.py "$(find "$D/tl" -name '*kernel_trace.csv' | head -1)" > "$D/timeline.txt" 2>&1
  find "$D/tl" -name '*.csv' -delete
  tail -12 "$D/timeline.txt"
}

step_e2e() {
  timeout -k 10 900 python3 tools/e2e_bench.py $E2E_ARGS > "$D/e2e.json" 2> "$D/e2e.err"
  local rc=$?
  tail -3 "$D/e2e.json"
  return $rc
}

for s in "$@"; do
  echo "### $s"
  case "$s" in
    test) step_test ;;
    tests=*) step_tests "${s#tests=}" ;;
    bench) step_bench ;;
    prof) step_prof ;;
    pmc) step_pmc ;;
    ab) step_ab ;;
    timeline) step_timeline ;;
    e2e) step_e2e ;;
    *) echo "unknown step $s"; false ;;
  esac
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "step $s failed rc=$rc: stopping"
    exit $rc
  fi
done
