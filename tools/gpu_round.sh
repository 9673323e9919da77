#!/bin/bash
# One gpurun call: GPU parity tests, smoke, bench, rocprofv3 kernel trace.
# Usage (on the GPU box, from the repo root): bash tools/gpu_round.sh [tests] [smoke] [bench] [prof]
# Every GPU step has its own time limit; a crash/timeout (rc > 1) ends the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
want() { [ $# -eq 0 ] && return 0; for a in $ARGS; do [ "$a" = "$1" ] && return 0; done; return 1; }
ARGS="$*"
[ -z "$ARGS" ] && ARGS="tests smoke bench prof"
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }

if want tests; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -n 4 gpurun_out/pytest_gpu.log; check $rc pytest
fi
if want smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; tail -n 2 gpurun_out/smoke.log; check $rc smoke
fi
if want bench; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?; tail -n 2 gpurun_out/bench.log; check $rc bench
fi
if want prof; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/prof_${TAG} -o kt -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} \
      > gpurun_out/prof_${TAG}.log 2>&1
  rc=$?; tail -n 2 gpurun_out/prof_${TAG}.log; check $rc rocprof
  find gpurun_out/prof_${TAG} -name "*stats*" | head
fi
exit 0
