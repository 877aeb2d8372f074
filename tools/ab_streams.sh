set -e
mkdir -p gpurun_out/ab
for r in 1 2; do for L in 4 4f 5 6 13; do
  TB_STREAMS=$L timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/ab/b_${L}_$r.log 2>&1
  echo "$r $L $(tail -1 gpurun_out/ab/b_${L}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done; done
