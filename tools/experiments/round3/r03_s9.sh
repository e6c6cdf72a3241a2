set -o pipefail
export TMPDIR=/tmp
PEMP_NO_UPD_FUSE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s9_mpn_noupd.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s9_mpn.log 2>&1 && \
PEMP_NO_UPD_FUSE=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03s9_noupd -o run -- \
  python bench.py --no-cpu-baseline --no-roofline --steps 20 --streams 1 > gpurun_out/r03s9_noupd.log 2>&1 && \
PEMP_NO_UPD_FUSE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --streams 1 > gpurun_out/r03s9_c3_noupd.json 2>/dev/null && \
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --streams 1 > gpurun_out/r03s9_c3.json 2>/dev/null
