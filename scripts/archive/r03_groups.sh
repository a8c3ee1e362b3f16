# bench shape sweep (sequences per GPU / stream groups), headline legs only
set -o pipefail
mkdir -p gpurun_out
Q="--no-cpu-baseline --lba-batch 0 --pcie-steps 0 --single-stream-steps 0 --budget-steps 0 --isolated-steps 0"
for g in ${GROUPS_LIST:-1 2 4}; do
  timeout -k 10 300 python bench.py $Q --groups $g ${EXTRA} > gpurun_out/${1:-gs}_g$g.json 2> gpurun_out/${1:-gs}_g$g.err || exit 10
done
