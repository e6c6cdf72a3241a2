# round 4, call v: rocprofv3 kernel stats of one-stream bench runs (c3, c3knn10): per-kernel averages without the
# second stream's contention, next to the line's own event-timed roofline of the same command
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in c3 c3knn10; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04v_${wl} -o run -- \
    python bench.py --workload $wl --streams 1 --no-cpu-baseline --steps 20 > gpurun_out/r04v_${wl}.json 2> gpurun_out/r04v_${wl}.err || exit 1
  echo "$wl ok"
done
