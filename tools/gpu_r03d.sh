#!/bin/bash
# r03d: KB normal-equations sweep (37-sum KB layout), RadTan config-4 tail
# diagnosis, NE parity tests.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03d}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_solver.py tests/test_gpu_configs.py -k "normal or conversion or config3 or lm" -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
check $? pytest; tail -n 3 gpurun_out/${TAG}_pytest.log
NE_MODELS=2,3 timeout -k 10 300 python tools/bench_configs.py --configs 3ne > gpurun_out/${TAG}_ne.log 2>&1
check $? ne_sweep; cat gpurun_out/${TAG}_ne.log
timeout -k 10 300 python tools/diag_radtan_tail.py > gpurun_out/${TAG}_radtan_tail.log 2>&1
check $? radtan_tail; cat gpurun_out/${TAG}_radtan_tail.log
echo done
