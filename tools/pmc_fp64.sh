#!/bin/bash
# Counter evidence for the FP64-bound kernels (tools/fp64_kernels.py):
# one kernel-trace --stats pass, then one rocprofv3 --pmc pass per counter
# group (kernel trace only alongside, as MI355X_MICROARCH.md prescribes).
# Each pass has its own SIGKILL time limit; a failure ends the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
DRV=${DRV:-"tools/fp64_kernels.py --reps 3"}
timeout -s KILL 60 rocprofv3 -L > gpurun_out/rocprof_counters_list.txt 2>&1
echo "list rc=$?"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
   -d gpurun_out/fp64_${TAG}_kt -o kt -- python3 $DRV > gpurun_out/fp64_${TAG}_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -ne 0 ] && { tail -n 5 gpurun_out/fp64_${TAG}_kt.log; exit $rc; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_TRANS_F64 SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LEVEL_WAVES SQ_INSTS_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
     -d gpurun_out/fp64_${TAG}_pmc$i -o pmc -- python3 $DRV > gpurun_out/fp64_${TAG}_pmc$i.log 2>&1
  rc=$?; echo "pmc[$grp] rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 gpurun_out/fp64_${TAG}_pmc$i.log; exit $rc; fi
done
exit 0
