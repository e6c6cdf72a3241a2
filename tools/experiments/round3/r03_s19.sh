set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03s19_c3.json 2> gpurun_out/r03s19_c3.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --workload c2 > gpurun_out/r03s19_c2.json 2> gpurun_out/r03s19_c2.err || exit 1
