#!/bin/bash
# r03f: interval-certificate random-camera tests, write-pass NT variant.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03f}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_kb_keep_boundary.py tests/test_capi.py -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
check $? pytest; tail -n 5 gpurun_out/${TAG}_pytest.log
VARIANTS=seg,seg_w5,seg_w3 timeout -k 10 500 python tools/diag_sample.py > gpurun_out/${TAG}_diag_sample.log 2>&1
check $? diag_sample; grep model gpurun_out/${TAG}_diag_sample.log | cut -c1-250
echo done
