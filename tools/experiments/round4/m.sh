# round 4, call m: stage-1 NMS variants (1 column per lane vs 4, bands per wave, ranking cost) on c3; a failing
# detection edge case against the oracle (quads vs strips build); phase clocks of the fused select + emit stage
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/debug/detect_case.py 37 8 1 > gpurun_out/r04m_case.txt 2>&1
echo "case rc=$?"
PEMP_LIB=$PWD/build_ab/libpemp_strips.so timeout -k 10 120 python tools/debug/detect_case.py 37 8 1 > gpurun_out/r04m_case_strips.txt 2>&1
echo "case strips rc=$?"
AB_ARGS="--workload c3" timeout -k 10 900 bash tools/ab.sh default strips norank b2 b8 norank_b8
PEMP_LIB=$PWD/build_ab/libpemp_clocks.so timeout -k 10 200 python bench.py --workload c3 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r04m_clocks.log 2>&1
echo "clocks rc=$?"
