# Isolated NMS timing (tools/nms_bench.py, back-to-back pemp_detect at c3): strip kernel vs quad kernel and quad
# variants (build_ab/libpemp_<v>.so), then a rocprofv3 kernel trace of both kernels.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06qi}
for round in 1 2; do
  PEMP_NMS_QUAD=0 timeout -k 10 120 python tools/nms_bench.py c3 || exit 1
  PEMP_NMS_QUAD=1 timeout -k 10 120 python tools/nms_bench.py c3 || exit 1
  for v in ${VARIANTS:-}; do
    PEMP_LIB=$PWD/build_ab/libpemp_$v.so PEMP_NMS_QUAD=1 timeout -k 10 120 python tools/nms_bench.py c3 | sed "s/^/$v /" || exit 1
  done
done
for q in 0 1; do
  PEMP_NMS_QUAD=$q timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof$q -o k -- python tools/nms_bench.py c3 20 > gpurun_out/${T}_prof$q.log 2>&1 || exit 1
  find gpurun_out/${T}_prof$q -name "*kernel_stats.csv" -exec grep -h -E "nms_|plane_emit" {} \; | cut -c1-200
done
find gpurun_out -type f \( -name "*kernel_trace.csv" -o -name "*.db" \) -size +1M -delete
