#!/bin/bash
# GPU validation run used with gpurun: tests first; a crash/timeout stops everything after it.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 ${TB_TEST_TIMEOUT:-600} python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
src=$?
tail -5 gpurun_out/smoke.log
echo "smoke rc=$src"
exit $(( rc != 0 ? rc : src ))
