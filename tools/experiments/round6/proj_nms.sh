# round 6: the separable projected NMS loader with buffer loads, a static flip and one ds_read2 per map and row
# (default) vs round 5's loader (build_ab/libpemp_projold.so): the projected / detection GPU tests, then the
# frontend leg (detection alone, both arms) alternating
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06j}
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread \
    -k "projected or detection or nms or frontend" > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
echo "tests $(tail -1 gpurun_out/${T}_tests.log)"
for v in ${VARIANTS:-default projold default projold}; do
  if [ $v = default ]; then unset PEMP_LIB; else export PEMP_LIB=$PWD/build_ab/libpemp_$v.so; fi
  timeout -k 10 200 python tools/frontend_detect.py c3 > gpurun_out/${T}_front_$v.json 2> gpurun_out/${T}_front_$v.err || { tail -20 gpurun_out/${T}_front_$v.err; exit 1; }
  echo "$v $(tail -1 gpurun_out/${T}_front_$v.json)"
done
unset PEMP_LIB
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python tools/frontend_detect.py c3 > gpurun_out/${T}_prof.log 2>&1 || exit 1
echo prof done
