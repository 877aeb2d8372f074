#!/bin/bash
# Config 5 bench + phase profile (tools/gpu_c5.sh), then PMC passes on the headline bench.
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/gpu_c5.sh || exit $?
TB_PROF_STEPS=2 bash tools/profile_pmc.sh || exit $?
