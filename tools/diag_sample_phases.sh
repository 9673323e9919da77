#!/bin/bash
# sample_points phase split (KB, 1e8 cells): the production kernel, a build
# without the output stores (ACM_DIAG_SAMPLE=1) and one without the
# unprojection (=2), one with neither (=3: look-back and compaction only)
# and one without the look-back too (=6), each under a rocprofv3 kernel trace.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r02}
for lib in ${LIBS:-libacm libacm_diag1 libacm_diag2 libacm_diag3 libacm_diag6}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/phase_${TAG}_$lib -o kt -- \
    python3 tools/fp64_kernels.py --only sample_kb --reps 5 --lib apex-camera-models_amd/lib/$lib.so \
    > gpurun_out/phase_${TAG}_$lib.log 2>&1 || exit $?
  grep kernel gpurun_out/phase_${TAG}_$lib.log
done
