#!/bin/bash
# Normal equations with the prologue loads kept in the loop's issue order:
# parity over every knob cell, then the sweep over every model.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03p}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "normal" -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
check $? pytest; tail -n 3 gpurun_out/${TAG}_pytest.log
timeout -k 10 600 python3 -u tools/bench_configs.py --configs 3ne > gpurun_out/${TAG}_ne_all.log 2>&1
check $? ne_sweep; grep -o '"model": "[A-Za-z]*".*"best": "[a-z0-9-]*", "Mpoints_per_s": [0-9.]*, "GBps": [0-9.]*' gpurun_out/${TAG}_ne_all.log
echo done
