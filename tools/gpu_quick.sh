#!/bin/bash
# Quick GPU iteration: the GPU test suite (optional), then sample_points A/B.
# Every step has its own time limit; a crash or timeout (rc > 1) ends it.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03a}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
if [ -n "${TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest ${TESTS} -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest_gpu.log 2>&1
check $? pytest; tail -n 3 gpurun_out/${TAG}_pytest_gpu.log
fi
if [ -n "${SAMPLE:-}" ]; then
MODELS=${SAMPLE} timeout -k 10 300 python tools/diag_sample.py > gpurun_out/${TAG}_diag_sample.log 2>&1
check $? diag_sample; cat gpurun_out/${TAG}_diag_sample.log | grep model
fi
if [ -n "${PROF:-}" ]; then
MODELS=${PROF} VARIANTS=-1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_sprof -o kt \
  -- python3 tools/diag_sample.py > gpurun_out/${TAG}_sprof.log 2>&1
check $? rocprof_sample
fi
echo done
