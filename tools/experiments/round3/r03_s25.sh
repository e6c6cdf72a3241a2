# node_rows: embedding / heads weights by LDS-DMA (MPN parity, then kernel stats + bench c3)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_mpn.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s25_mpn.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03s25_stats -o run -- python bench.py --steps 50 --warmup 10 --streams 1 > gpurun_out/r03s25_prof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r03s25_c3.json 2> gpurun_out/r03s25_c3.err || exit 1
