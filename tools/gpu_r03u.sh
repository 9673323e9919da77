#!/bin/bash
# Column-parallel normal-equations epilogue: NE parity, the LM (host-polled
# flag path) and distributed tests, then the NE sweep and the config-3 LM
# against lib/libacm_ab.so (a build of the previous commit).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03u}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_solver.py tests/test_gpu_distributed.py tests/test_gpu_configs.py -k "normal or lm or solver or convert or distributed or config3" -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
check $? pytest; tail -n 3 gpurun_out/${TAG}_pytest.log
for rep in 1 2; do
  for lib in libacm.so libacm_ab.so; do
    ACM_LIB_PATH=$PWD/apex-camera-models_amd/lib/$lib NE_MODELS=0,2,3 timeout -k 10 300 python3 -u tools/bench_configs.py --configs 3ne,3 > gpurun_out/${TAG}_${lib}_${rep}.log 2>&1
    rc=$?; echo "$lib rep $rep rc=$rc"
    grep -o '"model": "[A-Za-z]*".*"w0u0n-1": [0-9.]*' gpurun_out/${TAG}_${lib}_${rep}.log
    grep -o '"convert_s": [0-9.]*' gpurun_out/${TAG}_${lib}_${rep}.log
    if [ $rc -gt 1 ]; then exit $rc; fi
  done
done
echo done
