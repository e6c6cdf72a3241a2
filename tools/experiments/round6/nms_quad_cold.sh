# Isolated NMS timing with the Infinity Cache (MALL) evicted between calls (tools/nms_bench.py *_cold_us) and back to
# back: the strip kernel (PEMP_NMS_QUAD=0), the quad kernel, quad variants (build_ab/libpemp_<v>.so).
set -o pipefail
export TMPDIR=/tmp
for round in 1 2; do
  PEMP_NMS_QUAD=0 timeout -k 10 120 python tools/nms_bench.py c3 || exit 1
  PEMP_NMS_QUAD=1 timeout -k 10 120 python tools/nms_bench.py c3 || exit 1
  for v in ${VARIANTS:-}; do
    PEMP_LIB=$PWD/build_ab/libpemp_$v.so PEMP_NMS_QUAD=1 timeout -k 10 120 python tools/nms_bench.py c3 | sed "s/^/$v /" || exit 1
  done
done
# host time of the bench step (pipelined server loop, c2 and c3)
for wl in c2 c3; do
  timeout -k 10 200 python tools/step_host_timing.py $wl 300 bench > gpurun_out/r06h_host_$wl.log 2>&1 || { tail -5 gpurun_out/r06h_host_$wl.log; exit 1; }
  head -30 gpurun_out/r06h_host_$wl.log
done
