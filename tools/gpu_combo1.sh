#!/bin/bash
cd "$(dirname "$0")/.."
bash tools/gpu_lid3.sh || exit 1
bash tools/gpu_sweep3.sh
