# bench (headline legs only) under values of one environment variable: ab_env.sh TAG VAR v1 v2 ...
set -o pipefail
mkdir -p gpurun_out
Q="--no-cpu-baseline --lba-batch 0 --pcie-steps 0 --single-stream-steps 0 --budget-steps 0 --isolated-steps 0"
T=$1; V=$2; shift 2
for v in "$@"; do
  env $V=$v timeout -k 10 300 python bench.py $Q > gpurun_out/${T}_$v.json 2> gpurun_out/${T}_$v.err || exit 11
done
