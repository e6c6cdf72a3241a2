# round 5, call t: the embedding with two tiles per wave iteration (edge_embed2_kernel, 8 or 12 waves per workgroup)
# against the one-tile kernel (PEMP_EMBED2=0): MPN parity (goldens, oracle, determinism), per-shape times
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_mpn.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r05t_mpn_tests.log 2>&1
rc=$?; echo "mpn tests rc=$rc $(tail -1 gpurun_out/r05t_mpn_tests.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r05t_mpn_tests.log | head; exit 1; }
for v in one w8 w12; do
  case $v in one) envs="PEMP_EMBED2=0";; w8) envs="PEMP_EMBED2=1";; w12) envs="PEMP_EMBED2=1 PEMP_LIB=$PWD/build_ab/v_embed12/libpemp.so";; esac
  for wl in c3 c3knn10 c2; do
    env $envs timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05t_${v}_${wl} -o run -- \
        python bench.py --workload $wl --profile-steps --steps 20 --warmup 5 > gpurun_out/r05t_${v}_${wl}.log 2>&1 || exit 1
    python tools/trace_step_stats.py gpurun_out/r05t_${v}_${wl}/run_kernel_trace.csv 25 > gpurun_out/r05t_${v}_${wl}.md || exit 1
    echo "$v $wl: $(grep -E 'embed' gpurun_out/r05t_${v}_${wl}.md | grep -v image | head -1)"
  done
done
# the finishing chained on the grouping thread (GroupingJob.then): pose parity, the c3 e2e leg
timeout -k 10 400 python -u -m pytest tests/test_gpu_pose.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r05t_pose_tests.log 2>&1
rc=$?; echo "pose tests rc=$rc $(tail -1 gpurun_out/r05t_pose_tests.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r05t_pose_tests.log | head; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05t_c3.json 2> gpurun_out/r05t_c3.err || exit 1
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r05t_c3.json').read().strip().splitlines()[-1])
print('c3', d['value'], d.get('value_serial_steps'), json.dumps(d['e2e']))
PY
