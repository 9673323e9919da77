#!/bin/bash
# SQ-level counters (occupancy, VALU vs wait) for the project kernels of
# selected models: one counter group per rocprofv3 pass, kernel trace only.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-sq}
MODELS=${MODELS:-kb,ds}
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
           "SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LEVEL_WAVES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_TRANS_F64 SQ_THREAD_CYCLES_VALU SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
     -d gpurun_out/pmc_${TAG}_$i -o pmc -- python3 tools/sweep_project.py --rounds 1 --reps 2 \
     --models $MODELS --variants 1 --layouts aos --jac 1 > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?; echo "pmc[$grp] rc=$rc"
  if [ $rc -gt 1 ]; then tail -n 5 gpurun_out/pmc_${TAG}_$i.log; exit $rc; fi
done
exit 0
