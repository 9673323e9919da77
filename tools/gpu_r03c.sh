#!/bin/bash
# r03c: sample_points tests, write-pass variants for every model, and the
# kernel trace of the default segment path.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03c}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_kb_keep_boundary.py tests/test_gpu_parity.py tests/test_gpu_numerics_per_call.py tests/test_capi.py -k "sample or keep or cert or numerics or thread or tuning" -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
check $? pytest; tail -n 3 gpurun_out/${TAG}_pytest.log
VARIANTS=seg,seg_w1,seg_w3,seg_w4,seg_nocert,fused_r4 timeout -k 10 500 python tools/diag_sample.py > gpurun_out/${TAG}_diag_sample.log 2>&1
check $? diag_sample; grep model gpurun_out/${TAG}_diag_sample.log
MODELS=2,3,0,6 VARIANTS=seg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_sprof -o kt \
  -- python3 tools/diag_sample.py > gpurun_out/${TAG}_sprof.log 2>&1
check $? rocprof_sample
find gpurun_out/${TAG}_sprof -name "*kernel_stats.csv" -exec cat {} \; | grep -i "seg\|scan" | cut -c1-60,150-230
echo done
