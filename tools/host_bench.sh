#!/bin/bash
# Build + run the host assembly micro-benchmark; with PROFILE=1, under gprof.
set -e
cd "$(dirname "$0")/.."
srcs="csrc/host/devplan_build.cpp csrc/host/filters.cpp csrc/host/html.cpp csrc/host/json.cpp csrc/host/pipeline.cpp csrc/host/text.cpp"
flags="-O2 -std=c++17 -march=x86-64-v2"
[ -n "$PROFILE" ] && flags="$flags -pg -fno-omit-frame-pointer -fno-inline-functions"
g++ $flags -o build/host_bench tools/host_bench.cpp $srcs -licuuc -lpthread
cd build && ./host_bench "$@"
[ -n "$PROFILE" ] && gprof -b -p ./host_bench gmon.out | head -40 || true
