#!/bin/bash
# TokenCounter on the device: GPU tests (k_bpe_count vs host, device engine vs CPU oracle, the
# ICU-oracle net on hard documents), then the reference's default pipeline (config/pipeline_config.yaml,
# TokenCounter with a synthetic GPT-2-format tokenizer) with device counting, with host counting
# (TB_DEVICE_TOKENS=0), and without the TokenCounter step. Output gpurun_out/tok/.
cd "$(dirname "$0")/.."
OUT=gpurun_out/tok
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_bpe.py tests/test_gpu_e2e.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
python - <<'PY'
import yaml
d = yaml.safe_load(open("config/pipeline_config.yaml"))
d["pipeline"] = [s for s in d["pipeline"] if s["type"] != "TokenCounter"]
yaml.safe_dump(d, open("gpurun_out/tok/default_no_tc.yaml", "w"))
PY
for spec in "dev::config/pipeline_config.yaml" "host:TB_DEVICE_TOKENS=0:config/pipeline_config.yaml" "notc::gpurun_out/tok/default_no_tc.yaml"; do
  name=${spec%%:*}; rest=${spec#*:}; envs=${rest%%:*}; cfg=${rest#*:}
  env $envs timeout -k 10 400 python bench.py --steps ${TB_STEPS:-20} --warmup 3 --config $cfg --tokenizer synthetic > $OUT/b_$name.json 2> $OUT/b_$name.err || { tail -5 $OUT/b_$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_$name.json').read().strip().splitlines()[-1]); print('%-6s %.0f docs/s %.3f ms/step kept=%s cpu_ms/step=%s' % ('$name', d['value'], d['ms_per_step'], d.get('kept'), d.get('host_cpu_ms_per_step')))"
done
