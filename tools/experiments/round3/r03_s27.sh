# node_rows heads: layer weights read from LDS ahead of the MFMA chains (MPN parity, kernel stats, bench c3)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_mpn.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s27_mpn.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03s27_stats -o run -- python bench.py --steps 50 --warmup 10 --streams 1 > gpurun_out/r03s27_prof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r03s27_c3.json 2> gpurun_out/r03s27_c3.err || exit 1
