#!/bin/bash
# project+J (and project only) bench line for every model at 10M points
# (bench.py's own timing), one process per cell.
set -u
mkdir -p gpurun_out
for m in pinhole radtan kb ds ucm eucm fov; do
  timeout -k 10 120 python bench.py --model $m --no-cpu-baseline --steps 30 > gpurun_out/sweep_$m.log 2>&1 || exit $?
  tail -n 1 gpurun_out/sweep_$m.log
  timeout -k 10 120 python bench.py --model $m --no-jacobian --no-cpu-baseline --steps 30 > gpurun_out/sweep_${m}_noj.log 2>&1 || exit $?
  tail -n 1 gpurun_out/sweep_${m}_noj.log
done
