#!/bin/bash
# FOV grid: record kernel with whole-record prefetch -- bit identity vs the
# LDS kernel, then the A/B at config scale.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03o}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py -k "fov" -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
check $? pytest; tail -n 3 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python3 -u tools/bench_configs.py --configs fov > gpurun_out/${TAG}_fov.log 2>&1
check $? fov; tail -n 2 gpurun_out/${TAG}_fov.log | cut -c1-400
echo done
