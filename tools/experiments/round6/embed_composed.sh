# round 6: (1) the edge embedding composed with the first edge-MLP layer (Q0, R0 straight from h3) and (2) the
# cross-lane sums on v_permlane16/32_swap + DPP instead of ds_bpermute shuffles (edge-pass attention / head dots,
# NMS unit counts). MPN + graph GPU tests, then isolated-MPN A/B against the same tree without (1)
# (build_ab/libpemp_nocomp.so) and without (2) in mpn.hip (noperm), and c3 bench lines with and without (2) in
# detect.hip (nmsnoperm) for the NMS kernel time.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06c}
timeout -k 10 500 python -u -m pytest tests/test_gpu_mpn.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
echo "tests $(tail -1 gpurun_out/${T}_tests.log)"
for wl in c3 c3knn10 c2; do
  timeout -k 10 300 python tools/mpn_ab.py --workload $wl --iters 40 default nocomp noperm default nocomp noperm > gpurun_out/${T}_ab_$wl.txt 2>&1 || exit 1
  cat gpurun_out/${T}_ab_$wl.txt
done
AB_ARGS="--no-backbone" timeout -k 10 600 bash tools/ab.sh default nmsnoperm default nmsnoperm 2>&1 | tee gpurun_out/${T}_nms_ab.txt
