#!/bin/bash
# KB normal equations: wave-split accumulation A/B (ACM_TUNE_NE_SPLIT) and
# its parity; the per-call-numerics thread test after the stream fix.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03h}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
check $? pytest; tail -n 3 gpurun_out/${TAG}_pytest.log
NE_MODELS=2 timeout -k 10 300 python3 -u tools/bench_configs.py --configs 3ne > gpurun_out/${TAG}_ne_kb.log 2>&1
check $? ne_sweep; cat gpurun_out/${TAG}_ne_kb.log | tail -n 3
NE_MODELS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_neprof -o kt \
  -- python3 tools/bench_configs.py --configs 3ne > gpurun_out/${TAG}_neprof.log 2>&1
check $? ne_prof
grep -h "normal_eq\|ne_kb_split" gpurun_out/${TAG}_neprof/*kernel_stats.csv | cut -c1-90,150-230
echo done
