# round 4, call q: capacity-mode MPN A/B (bind_mpn on / off), c2 and c3, alternating to see the box's noise
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ARGS="--workload c2 --steps 100" timeout -k 10 600 bash tools/ab_env.sh c2cap: c2nocap:PEMP_NO_CAP_MPN=1 c2cap2: c2nocap2:PEMP_NO_CAP_MPN=1
AB_ARGS="--workload c3 --steps 30" timeout -k 10 600 bash tools/ab_env.sh c3cap: c3nocap:PEMP_NO_CAP_MPN=1
