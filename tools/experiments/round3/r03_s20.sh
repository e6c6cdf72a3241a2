set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s20_mpn.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --streams 1 > gpurun_out/r03s20_c3.json 2> gpurun_out/r03s20_c3.err || exit 1
PEMP_LIB=build_ab/libpemp_base.so timeout -k 10 300 python bench.py --no-cpu-baseline --streams 1 > gpurun_out/r03s20_c3b.json 2> gpurun_out/r03s20_c3b.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03s20_stats -o run -- \
  python bench.py --no-cpu-baseline --no-roofline --steps 20 --streams 1 > gpurun_out/r03s20_stats.log 2>&1
