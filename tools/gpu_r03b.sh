#!/bin/bash
# r03b: segment sample_points kernel breakdown (rocprofv3 kernel trace),
# config 4 round trip after the NaN early-outs, config-4/5 scale tests.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03b}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
MODELS=2,3,0 VARIANTS=-1,-2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_sprof -o kt \
  -- python3 tools/diag_sample.py > gpurun_out/${TAG}_sprof.log 2>&1
check $? rocprof_sample
grep model gpurun_out/${TAG}_sprof.log
find gpurun_out/${TAG}_sprof -name "*kernel_stats.csv" -exec cat {} \; | grep -i "seg\|scan\|Name" | cut -c1-200
timeout -k 10 300 python tools/bench_configs.py --configs 4 > gpurun_out/${TAG}_configs.log 2>&1
check $? configs4
grep -o '"model": "[a-z_]*".*"unproject_GBps": [0-9.]*' gpurun_out/${TAG}_configs.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest_cfg.log 2>&1
check $? pytest_cfg; tail -n 3 gpurun_out/${TAG}_pytest_cfg.log
echo done
