#!/bin/bash
# After making the speculative segment path RadTan's default: the GPU suite,
# smoke, the bench line, one sample_points kernel trace of every model, and
# the FOV grid kernel A/B (per-point records vs LDS staging).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03n}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
check $? pytest; tail -n 3 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
check $? smoke; tail -n 1 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python3 -u bench.py > gpurun_out/${TAG}_bench.log 2>&1
check $? bench; tail -n 1 gpurun_out/${TAG}_bench.log | cut -c1-300
VARIANTS=seg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_sprof -o kt \
  -- python3 tools/diag_sample.py > gpurun_out/${TAG}_sample.log 2>&1
check $? sample_prof; tail -n 1 gpurun_out/${TAG}_sample.log | cut -c1-600
timeout -k 10 300 python3 -u tools/bench_configs.py --configs fov > gpurun_out/${TAG}_fov.log 2>&1
check $? fov; tail -n 2 gpurun_out/${TAG}_fov.log | cut -c1-400
echo done
