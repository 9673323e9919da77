#!/bin/bash
# KB normal equations: prefetch depth (NE_UNROLL 4, 5) A/B and parity.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03i}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -k "normal or sharded" -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
check $? pytest; tail -n 3 gpurun_out/${TAG}_pytest.log
NE_MODELS=2 timeout -k 10 300 python3 -u tools/bench_configs.py --configs 3ne > gpurun_out/${TAG}_ne_kb.log 2>&1
check $? ne_sweep; tail -n 1 gpurun_out/${TAG}_ne_kb.log
NE_MODELS=2 timeout -k 10 300 python3 -u tools/bench_configs.py --configs 3ne > gpurun_out/${TAG}_ne_kb2.log 2>&1
check $? ne_sweep2; tail -n 1 gpurun_out/${TAG}_ne_kb2.log
echo done
