#!/bin/bash
# RadTan sample_points on drop cameras: parity of every path,
# then auto / speculative / single pass on cameras with and without drops
# (tools/diag_sample_drops.py).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03s}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -k "sample" -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
check $? pytest; tail -n 3 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python3 -u tools/diag_sample_drops.py > gpurun_out/${TAG}_drops.log 2>&1
check $? drops; grep camera gpurun_out/${TAG}_drops.log
echo done
