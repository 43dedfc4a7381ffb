#!/bin/bash
# Weight-gradient limiter study: per-layer solo times on whole-chip grids, the RN_DIAG
# removal bits of wgrad_big_kernel (rn_set_tuning 6: 1 no epilogue, 2 no loop DMAs, 4 no waits/barriers),
# and SQ counters of representative layers. usage: bash tools/runs/wgrad_diag.sh TAG [bench]
tag=$1; shift
set -o pipefail
mkdir -p gpurun_out
if [ "$1" = bench ]; then
  timeout -k 10 200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_c2.log 2>&1 || exit $?
fi
timeout -k 10 200 env RN_TUNE=21=100 python tools/conv_bench.py --only wgrad --iters 20 > gpurun_out/${tag}_wg100.log 2>&1 || exit $?
timeout -k 10 200 python tools/conv_bench.py --only wgrad --iters 20 > gpurun_out/${tag}_wg45.log 2>&1 || exit $?
for bits in 0 1 2 4 6 7; do
  timeout -k 10 200 env RN_LIB_PATH=resnet.mxnet_amd/rn/librn_diag.so RN_TUNE=21=100,6=$bits python tools/conv_bench.py --only wgrad --iters 10 > gpurun_out/${tag}_diag_$bits.log 2>&1 || exit $?
done
for f in stage3_unit2_conv2 stage2_unit2_conv1 stage4_unit2_conv2; do
  RN_TUNE=21=100 timeout -k 10 400 bash tools/pmc_conv.sh ${tag}_$f --filter $f --only wgrad --iters 10 > gpurun_out/${tag}_pmc_$f.log 2>&1 || exit $?
  python tools/pmc_conv_summary.py gpurun_out/pmcc_${tag}_$f > gpurun_out/${tag}_pmcsum_$f.txt 2>&1
done
