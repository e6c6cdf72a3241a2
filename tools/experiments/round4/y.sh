# round 4, call y: NMS two units ahead (pf2) vs one (default), c3 one stream, alternating
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ARGS="--workload c3 --steps 30 --streams 1" timeout -k 10 600 bash tools/ab.sh default pf2 default pf2
