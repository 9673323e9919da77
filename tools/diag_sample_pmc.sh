set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_undistort.py -x -q --timeout 120 --timeout-method thread -rf > gpurun_out/pytest_exact_r02b.log 2>&1
rc=$?; tail -n 5 gpurun_out/pytest_exact_r02b.log; [ $rc -gt 1 ] && exit $rc
for v in 0 1 2 3; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/samp_r02b_v$v -o kt -- python3 tools/fp64_kernels.py --only sample_kb --reps 5 --sample-fused $v > gpurun_out/samp_r02b_v$v.log 2>&1 || exit $?
done
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_INSTS_LDS SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LEVEL_WAVES SQ_INSTS_SMEM"; do
  i=$((${i:-0}+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/samp_r02b_pmc$i -o pmc -- python3 tools/fp64_kernels.py --only sample_kb,kb_unproject --reps 3 > gpurun_out/samp_r02b_pmc$i.log 2>&1 || exit $?
done
echo done
