# round 5, call a: GPU suite with the graph-capture fixes; the asm-vs-compiler scan check on the bf16x3 goldens
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05a_gpu_tests.log 2>&1
echo "suite rc=$? $(tail -1 gpurun_out/r05a_gpu_tests.log)"
PEMP_LIB=$PWD/build_ab/libpemp_asmchk.so timeout -k 10 120 python -u -m pytest tests/test_gpu_mpn.py -q -s -k "golden and attn and bf16x3" --timeout 100 --timeout-method thread > gpurun_out/r05a_asmchk.log 2>&1
echo "asmchk rc=$? $(tail -1 gpurun_out/r05a_asmchk.log)"
grep -c ASMCHK gpurun_out/r05a_asmchk.log || true
# host GAEC on the box's cores (no GPU): thread counts and the pool's spin window
for sp in 0 2000; do for t in 1 4 8 16; do
  PEMP_POOL_SPIN_US=$sp timeout -k 5 60 python -u tools/gaec_bench.py 8 153 9 $t 50 | sed "s/^/spin=$sp /"
done; done
PEMP_GAEC_EXACT=1 timeout -k 5 60 python -u tools/gaec_bench.py 8 153 9 1 20 | sed "s/^/exact /"
timeout -k 5 60 python -u tools/gaec_bench.py 1 502 36 1 20
PEMP_GAEC_EXACT=1 timeout -k 5 60 python -u tools/gaec_bench.py 1 502 36 1 10 | sed "s/^/exact /"
# MFMA utilisation calibration: dense f16 MFMA on every SIMD, events, then the SQ / GRBM counters
timeout -k 5 60 build_ab/mfma_peak 20000 1 | tee gpurun_out/r05a_mfma_peak.json
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/r05a_mfma_pmc -o pmc -- build_ab/mfma_peak 20000 1 > gpurun_out/r05a_mfma_pmc.log 2>&1
echo "mfma pmc rc=$?"
