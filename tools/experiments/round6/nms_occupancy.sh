# round 6: the NMS strip kernel at 6 waves per SIMD (amdgpu_waves_per_eu(6): <= 80 VGPRs, NMS_PER_CU 6) against the
# default 5 (83 VGPRs): graph GPU tests on the variant, then c3 bench lines alternating (tools/ab.sh)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06f}
PEMP_LIB=$PWD/build_ab/libpemp_nms6.so timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
echo "tests (nms6) $(tail -1 gpurun_out/${T}_tests.log)"
AB_ARGS="--no-backbone" timeout -k 10 900 bash tools/ab.sh default nms6 default nms6 default nms6 2>&1 | tee gpurun_out/${T}_nms_ab.txt
