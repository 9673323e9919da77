#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03g}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_numerics_per_call.py tests/test_gpu_kb_keep_boundary.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "sample or keep or cert or numerics or thread or config5" -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
check $? pytest; tail -n 3 gpurun_out/${TAG}_pytest.log
MODELS=2 VARIANTS=seg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_sprof -o kt \
  -- python3 tools/diag_sample.py > gpurun_out/${TAG}_sample.log 2>&1
check $? sample_prof
grep -h "seg_\|scan" gpurun_out/${TAG}_sprof/*kernel_stats.csv | cut -c1-60,150-200
echo done
