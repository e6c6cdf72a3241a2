set -e
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --hip-runtime-trace --output-format csv -d gpurun_out/r03f_api -o run -- \
  python bench.py --no-cpu-baseline --no-roofline --steps 20 --streams 1 > gpurun_out/r03f_api.log 2>&1
python tools/api_report.py gpurun_out/r03f_api/run_hip_api_trace.csv > gpurun_out/r03f_api_report.md
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r03f_base.json 2>/dev/null
PEMP_LIB=build_ab/libpemp_nmspf2.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r03f_pf2.json 2>/dev/null
