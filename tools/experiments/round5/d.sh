# round 5, call d: is the asm-scan failure a race? determinism of the failing and passing builds; env bisection;
# the capacity-mode test alone and after the graph tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in asmall default; do
  if [ $lib = default ]; then unset PEMP_LIB; else export PEMP_LIB=$PWD/build_ab/libpemp_$lib.so; fi
  for envs in "X=0" "PEMP_SERIAL_PRELUDE=1" "PEMP_NO_GRAPHS=1"; do
    env $envs timeout -k 10 60 python -u tools/debug/determinism.py mpn_attn_t3 bf16x3 10 | sed "s/^/$lib $envs /"
  done
  timeout -k 10 60 python -u tools/debug/determinism.py mpn_attn_t3 f16x3 10 | sed "s/^/$lib /"
done
unset PEMP_LIB
timeout -k 10 200 python -u -m pytest tests/test_gpu_mpn.py -q -k "capacity_mode" --timeout 120 --timeout-method thread > gpurun_out/r05d_cap_alone.log 2>&1
echo "cap alone rc=$? $(tail -1 gpurun_out/r05d_cap_alone.log)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_mpn.py -q -k "capacity_mode or projected" --timeout 120 --timeout-method thread > gpurun_out/r05d_cap_graph.log 2>&1
echo "cap after graph rc=$? $(tail -1 gpurun_out/r05d_cap_graph.log)"
