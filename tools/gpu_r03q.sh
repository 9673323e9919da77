#!/bin/bash
# KB certified-ray polynomials: sample_points parity, then the 1e8-cell A/B
# against lib/libacm_ab.so (a build of the previous commit).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03q}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kb_keep_boundary.py tests/test_gpu_configs.py -k "sample or keep or config5 or 1e8" -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
check $? pytest; tail -n 3 gpurun_out/${TAG}_pytest.log
TAG=${TAG}_ab MODELS=2 VARIANTS=seg,fused_r4,spec CMD="python tools/diag_sample.py" bash tools/gpu_ab.sh
check $? ab
echo done
