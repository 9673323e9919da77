#!/bin/bash
# Round-3 measurement call, part A (tests, smoke, bench, its kernel trace and
# PMC traffic); part B is tools/gpu_round_r03b.sh.  Original description: GPU tests, smoke, bench line, rocprofv3 kernel
# trace of the bench, the headline PMC passes (traffic) + their summary, the
# FP64-kernel counter passes + summary, every SURVEY 8(a) row beside the
# oracle, configs 1/3/4/5, one sample_points kernel trace for every model,
# the RadTan config-4 diagnosis and the PCIe-inclusive rate.  Every step has
# its own time limit; a crash or timeout (rc > 1) ends the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03}
check() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi; }
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest_gpu.log 2>&1
check $? pytest; tail -n 2 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
check $? smoke; tail -n 1 gpurun_out/${TAG}_smoke.log
fi
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1
check $? bench; tail -c 600 gpurun_out/${TAG}_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o kt \
  -- python3 bench.py --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
check $? rocprof
TAG=${TAG} bash tools/pmc_round.sh > gpurun_out/${TAG}_pmc_round.log 2>&1
check $? pmc_round
python3 profiles/collect_pmc.py gpurun_out/pmc_${TAG} --workload kb_project_jacobian_f64_aos \
  --points 10000000 --algorithmic-bytes 1690000000 --out gpurun_out/${TAG}_pmc_kb_project_jacobian.json > /dev/null 2>&1
check $? collect_pmc
echo done
