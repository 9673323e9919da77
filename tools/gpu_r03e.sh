#!/bin/bash
# r03e: full GPU suite, FOV grid timing, one rocprofv3 kernel trace of
# sample_points for every model.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03e}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest_gpu.log 2>&1
check $? pytest; tail -n 3 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 300 python tools/bench_configs.py --configs fov > gpurun_out/${TAG}_fov.log 2>&1
check $? fov; cut -c1-400 gpurun_out/${TAG}_fov.log
VARIANTS=seg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_sprof -o kt \
  -- python3 tools/diag_sample.py > gpurun_out/${TAG}_sprof.log 2>&1
check $? rocprof_sample
grep model gpurun_out/${TAG}_sprof.log | cut -c1-200
echo done
