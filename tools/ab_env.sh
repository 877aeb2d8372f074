#!/bin/bash
# Interleaved A/B of environment settings on the headline bench (noise is +-2 ms/step between
# single runs): AB_A / AB_B are env assignments ("X=1 Y=2"), AB_N rounds, median ms/step each.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
export HSA_ENABLE_IPC_MODE_LEGACY=0
N=${AB_N:-3}
for r in $(seq 1 $N); do
  for tag in A B; do
    if [ $tag = A ]; then E="$AB_A"; else E="$AB_B"; fi
    env $E timeout -k 10 300 python bench.py --steps ${AB_STEPS:-12} --warmup 3 $AB_ARGS > gpurun_out/ab/${tag}_$r.log 2>&1 || { echo "run $tag $r failed"; tail -5 gpurun_out/ab/${tag}_$r.log; exit 1; }
  done
done
python3 - "$N" "$AB_A" "$AB_B" <<'PY'
import json, statistics, sys
n = int(sys.argv[1])
for tag, env in (("A", sys.argv[2]), ("B", sys.argv[3])):
    ms = [json.loads([l for l in open(f"gpurun_out/ab/{tag}_{r}.log") if l.startswith("{")][-1])["ms_per_step"] for r in range(1, n + 1)]
    print(f"{tag} [{env}] median {statistics.median(ms):.2f} ms/step  runs {ms}")
PY
