# A/B of the executor's stream placement (RN_SIDE_STREAM, RN_MAIN_STREAM, RN_MAIN_PRIORITY) with the
# all-reduce hooks on / off (RN_BENCH_ALLREDUCE); usage: bash tools/runs/env_ab.sh TAG "VAR=V ..." ...
set -o pipefail
tag=$1; shift
i=0
for spec in "$@"; do
  i=$((i+1))
  timeout -k 10 200 env $spec python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_$i.log 2>&1 || exit $?
  echo "$spec" >> gpurun_out/${tag}_$i.log
done
