#!/bin/bash
# PMC passes (one counter group per pass, kernel-trace only alongside, as the
# MI355X guide prescribes) over a short bench run of the headline workload.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
BA=${BENCH_ARGS:-"--steps 5 --warmup 1 --no-cpu-baseline --legs none"}
timeout -k 10 120 rocprofv3 -L > gpurun_out/rocprof_counters_list.txt 2>&1
echo "list rc=$?"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_32B_sum" ${EXTRA_PMC:-}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
     -d gpurun_out/pmc_${TAG}_$i -o pmc -- python3 bench.py $BA > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?; echo "pmc[$grp] rc=$rc"
  if [ $rc -gt 1 ]; then tail -n 5 gpurun_out/pmc_${TAG}_$i.log; exit $rc; fi
done
exit 0
