#!/bin/bash
# Round-3 measurement call, part B (FP64 counters, rows, configs, sample_points
# trace, RadTan config-4 diagnosis, KB normal equations, PCIe rate).  Original description: GPU tests, smoke, bench line, rocprofv3 kernel
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
TAG=${TAG} bash tools/pmc_fp64.sh > gpurun_out/${TAG}_pmc_fp64.log 2>&1
check $? pmc_fp64
python3 profiles/summarize_kernels.py gpurun_out/fp64_${TAG} --out gpurun_out/${TAG}_fp64_kernels.json > gpurun_out/${TAG}_fp64_kernels.md 2>&1
check $? summarize
timeout -k 10 400 python tools/bench_rows.py > gpurun_out/${TAG}_rows.log 2>&1
check $? rows
timeout -k 10 400 python tools/bench_configs.py --configs 1,3,4,5 > gpurun_out/${TAG}_configs.log 2>&1
check $? configs
VARIANTS=seg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_sprof -o kt \
  -- python3 tools/diag_sample.py > gpurun_out/${TAG}_sample.log 2>&1
check $? sample_prof
timeout -k 10 300 python tools/diag_radtan_tail.py > gpurun_out/${TAG}_radtan_tail.log 2>&1
check $? radtan_tail
NE_MODELS=2 timeout -k 10 300 python tools/bench_configs.py --configs 3ne > gpurun_out/${TAG}_ne_kb.log 2>&1
check $? ne_kb
timeout -k 10 300 python tools/bench_e2e.py > gpurun_out/${TAG}_e2e.log 2>&1
check $? e2e
echo done
