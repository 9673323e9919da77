#!/bin/bash
# A/B of lib/libacm.so against lib/libacm_ab.so (make -C apex-camera-models_amd ab AB=-D...)
# on one diagnostic command, interleaved twice.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ab}
CMD=${CMD:-"python tools/diag_sample.py"}
for rep in 1 2; do
  for lib in libacm.so libacm_ab.so; do
    ACM_LIB_PATH=$PWD/apex-camera-models_amd/lib/$lib timeout -k 10 300 $CMD > gpurun_out/${TAG}_${lib}_${rep}.log 2>&1
    rc=$?; echo "$lib rep $rc: $(grep -h '"model"' gpurun_out/${TAG}_${lib}_${rep}.log | cut -c1-160)"
    if [ $rc -gt 1 ]; then exit $rc; fi
  done
done
