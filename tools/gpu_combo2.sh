#!/bin/bash
cd "$(dirname "$0")/.."
bash tools/gpu_c4v.sh || exit 1
bash tools/gpu_long.sh
