# A/B of the in-tree library against experiments/librn_base.so (RN_LIB_PATH) in one call.
# usage: bash tools/runs/ab_lib.sh TAG "<tests -k expr or ->" "<conv_bench args or ->" MODEL [MODEL ...]
set -o pipefail
tag=$1; kexpr=$2; cb=$3; shift 3
if [ "$kexpr" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -k "$kexpr" -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || exit $?
fi
if [ "$cb" != "-" ]; then
  for lib in base new; do
    p=""; [ $lib = base ] && p=experiments/librn_base.so
    timeout -k 10 300 env RN_LIB_PATH=$p RN_LIB_ALLOW_MISMATCH=1 python tools/conv_bench.py $cb > gpurun_out/${tag}_cb_$lib.log 2>&1 || exit $?
  done
fi
for m in "$@"; do
  for lib in base new base new; do
    p=""; [ $lib = base ] && p=experiments/librn_base.so
    timeout -k 10 200 env RN_LIB_PATH=$p RN_LIB_ALLOW_MISMATCH=1 python bench.py --model $m --no-cpu-baseline --pcie-steps 0 >> gpurun_out/${tag}_${m}_$lib.log 2>&1 || exit $?
  done
done
