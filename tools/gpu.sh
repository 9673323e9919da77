#!/bin/bash
# The one GPU launcher (replaces the per-experiment tools/gpu_*.sh scripts of
# rounds 1-3).  Runs the named steps in order on the gpurun box, each under
# its own time limit, writing gpurun_out/<TAG>_<step>.*; a crash, abort or
# timeout (rc > 1) ends the script -- nothing more touches the GPU after it.
#
#   TAG=r04a bash tools/gpu.sh tests smoke bench prof pmc fp64 rows configs
#
# Steps:
#   tests[=ARGS]       pytest -m gpu over tests/ (or ARGS: files / -k expr)
#   smoke              __graft_entry__.smoke()
#   bench              python bench.py (the driver's default line)
#   prof               rocprofv3 kernel trace of bench.py (no CPU baseline)
#   pmc                headline PMC passes (FETCH/WRITE_SIZE, EA requests)
#                      + profiles/collect_pmc.py summary
#   fp64[=KERNELS]     counter passes over tools/fp64_kernels.py (--only
#                      KERNELS) + profiles/summarize_kernels.py
#   rows               tools/bench_rows.py (every SURVEY 8(a) row vs oracle)
#   configs[=LIST]     tools/bench_configs.py --configs LIST (default 1,3,4,5)
#   sample             rocprofv3 kernel trace of tools/probes.py sample
#   radtan_tail        tools/probes.py radtan_tail (config-4 pixels)
#   e2e                tools/bench_e2e.py (PCIe-inclusive rate)
#   run:NAME:CMD       any command (words split on '+'), output to <TAG>_NAME.log
#   kt:NAME:CMD        rocprofv3 kernel trace of a python3 CMD
#   ab:NAME:CMD        CMD alternately on lib/libacm.so and lib/libacm_ab.so, x2
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04}
O=gpurun_out
check() {
  local rc=$1 name=$2
  echo "$name rc=$rc"
  if [ "$rc" -gt 1 ]; then echo "stopping after $name"; exit "$rc"; fi
}
# counter groups of the fp64 step: one rocprofv3 pass each (slot limits of
# MI355X_MICROARCH.md: <= 8 SQ, 4 TCC (FETCH_SIZE uses 3), 4 TCP, 2 TA, 2 TD)
PMC_GROUPS=(
  "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_TRANS_F64 SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LEVEL_WAVES SQ_INSTS_LDS"
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
for step in "$@"; do
  name=${step%%[=:]*}
  arg=""
  [[ "$step" == *=* ]] && arg=${step#*=}
  case "$name" in
  tests)
    targs=${arg//+/ }
    timeout -k 10 900 python -u -m pytest ${targs:-tests} -m gpu -q --timeout 300 \
      --timeout-method thread -rf > $O/${TAG}_pytest_gpu.log 2>&1
    check $? tests; tail -n 2 $O/${TAG}_pytest_gpu.log ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1
    check $? smoke; tail -n 1 $O/${TAG}_smoke.log ;;
  bench)
    timeout -k 10 300 python bench.py > $O/${TAG}_bench.log 2>&1
    check $? bench; tail -c 700 $O/${TAG}_bench.log; echo ;;
  prof)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof -o kt \
      -- python3 bench.py --no-cpu-baseline > $O/${TAG}_prof.log 2>&1
    check $? prof ;;
  pmc)
    TAG=${TAG} bash tools/pmc_round.sh > $O/${TAG}_pmc_round.log 2>&1
    check $? pmc
    python3 profiles/collect_pmc.py $O/pmc_${TAG} --workload kb_project_jacobian_f64_aos \
      --kernel "k_project_al<acm::Tag<acm::KannalaBrandt>" \
      --points 10000000 --algorithmic-bytes 1690000000 \
      --out $O/${TAG}_pmc_kb_project_jacobian.json > $O/${TAG}_collect_pmc.log 2>&1
    check $? collect_pmc ;;
  fp64)
    DRV="tools/fp64_kernels.py --reps 3 ${arg:+--only $arg}"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $O/fp64_${TAG}_kt -o kt -- python3 $DRV > $O/fp64_${TAG}_kt.log 2>&1
    check $? fp64_kt
    i=0
    for grp in "${PMC_GROUPS[@]}"; do
      i=$((i+1))
      timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
        -d $O/fp64_${TAG}_pmc$i -o pmc -- python3 $DRV > $O/fp64_${TAG}_pmc$i.log 2>&1
      check $? "fp64_pmc$i"
    done
    python3 profiles/summarize_kernels.py $O/fp64_${TAG} --out $O/${TAG}_fp64_kernels.json \
      > $O/${TAG}_fp64_kernels.md 2>&1
    check $? summarize; cat $O/${TAG}_fp64_kernels.md ;;
  rows)
    timeout -k 10 400 python tools/bench_rows.py > $O/${TAG}_rows.log 2>&1
    check $? rows ;;
  configs)
    timeout -k 10 500 python tools/bench_configs.py --configs ${arg:-1,3,4,5} > $O/${TAG}_configs.log 2>&1
    check $? configs; grep -h '"config"' $O/${TAG}_configs.log | cut -c1-220 ;;
  sample)
    VARIANTS=seg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $O/${TAG}_sprof -o kt -- python3 tools/probes.py sample > $O/${TAG}_sample.log 2>&1
    check $? sample ;;
  radtan_tail)
    timeout -k 10 300 python tools/probes.py radtan_tail > $O/${TAG}_radtan_tail.log 2>&1
    check $? radtan_tail ;;
  e2e)
    timeout -k 10 300 python tools/bench_e2e.py > $O/${TAG}_e2e.log 2>&1
    check $? e2e ;;
  run|kt|ab)
    rest=${step#*:}
    sub=${rest%%:*}
    cmd=${rest#*:}
    cmd=${cmd//+/ }
    if [ "$name" = run ]; then
      timeout -k 10 500 $cmd > $O/${TAG}_${sub}.log 2>&1
      check $? "run:$sub"; tail -n 20 $O/${TAG}_${sub}.log
    elif [ "$name" = kt ]; then
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_${sub}_kt -o kt \
        -- python3 $cmd > $O/${TAG}_${sub}_kt.log 2>&1
      check $? "kt:$sub"
    else
      for rep in 1 2; do
        for lib in libacm.so libacm_ab.so; do
          ACM_LIB_PATH=$PWD/apex-camera-models_amd/lib/$lib timeout -k 10 300 $cmd \
            > $O/${TAG}_${sub}_${lib}_${rep}.log 2>&1
          check $? "ab:$sub:$lib:$rep"
        done
      done
    fi ;;
  *)
    echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
