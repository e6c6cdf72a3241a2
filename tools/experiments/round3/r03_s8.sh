set -o pipefail
export TMPDIR=/tmp
PEMP_NO_UPD_FUSE=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03s8_noupd -o run -- \
  python bench.py --no-cpu-baseline --no-roofline --steps 20 --streams 1 > gpurun_out/r03s8_noupd.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03s8_upd -o run -- \
  python bench.py --no-cpu-baseline --no-roofline --steps 20 --streams 1 > gpurun_out/r03s8_upd.log 2>&1
