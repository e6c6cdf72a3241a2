# round 5, call b: capacity-mode regression debug; asm-scan bisection variants on the bf16x3 goldens; GPU suite
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTHONPATH=$PWD timeout -k 10 120 python -u tools/debug/cap_mode_debug.py > gpurun_out/r05b_capdbg.log 2>&1
echo "capdbg rc=$?"; cat gpurun_out/r05b_capdbg.log | tail -20
for v in asmall asmall_drain asmall_vol asmall_tail; do
  PEMP_LIB=$PWD/build_ab/libpemp_$v.so timeout -k 10 120 python -u -m pytest tests/test_gpu_mpn.py -q -k "golden and attn and bf16x3" --timeout 100 --timeout-method thread > gpurun_out/r05b_$v.log 2>&1
  echo "$v rc=$? $(tail -1 gpurun_out/r05b_$v.log)"
done
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r05b_gpu_tests.log 2>&1
echo "suite rc=$? $(tail -1 gpurun_out/r05b_gpu_tests.log)"; grep FAILED gpurun_out/r05b_gpu_tests.log | head
timeout -k 5 60 build_ab/mfma_peak 20000 1 | tee gpurun_out/r05b_mfma_peak.json
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r05b_mfma_pmc -o pmc -- build_ab/mfma_peak 20000 1 > gpurun_out/r05b_mfma_pmc.log 2>&1
python tools/mfma_util.py gpurun_out/r05b_mfma_pmc/pmc_counter_collection.csv
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-include-regex 'edge_step|edge_embed|node_' --output-format csv -d gpurun_out/r05b_mfma_c3 -o pmc -- python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/r05b_mfma_c3.log 2>&1
python tools/mfma_util.py gpurun_out/r05b_mfma_c3/pmc_counter_collection.csv
