#!/bin/bash
# Speculative segment sample_points: parity (every path incl. 4, stress
# cameras with drops, shards), then the 1e8-cell A/B for RadTan and KB.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03m}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "sample_points" -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
check $? pytest; tail -n 3 gpurun_out/${TAG}_pytest.log
MODELS=1,2,0 VARIANTS=spec,fused_r4,seg timeout -k 10 300 python3 -u tools/diag_sample.py > gpurun_out/${TAG}_diag_sample.log 2>&1
check $? diag_sample; tail -n 5 gpurun_out/${TAG}_diag_sample.log
echo done
