#!/bin/bash
# LDS-DMA ring for the fused normal equations: parity over every knob cell
# (incl. the ring), ragged ring batches, then the NE sweep over every model.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03l}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "normal" -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
check $? pytest; tail -n 3 gpurun_out/${TAG}_pytest.log
timeout -k 10 600 python3 -u tools/bench_configs.py --configs 3ne > gpurun_out/${TAG}_ne_all.log 2>&1
check $? ne_sweep; grep -o '"model": "[A-Za-z]*".*' gpurun_out/${TAG}_ne_all.log
echo done
