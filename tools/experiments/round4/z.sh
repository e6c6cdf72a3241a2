# round 4, call z: size-gated node update fusion (default: separate at this size) vs always fused (sumall) on the published model
# (c3knn10, T=10: nine middle steps per forward), one stream, alternating
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ARGS="--workload c3knn10 --steps 20 --streams 1" timeout -k 10 600 bash tools/ab.sh default sumall default sumall
