# Round 6: the XPL data-gradient tile (rn_set_tuning 27) and the wgrad_big_kernel DMA / DIR change, against
# experiments/librn_base.so (the round-5 build) where a kernel has no key. usage: bash tools/runs/r06b_xpl.sh TAG
set -o pipefail
tag=${1:-r06b}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -k "bn_input_in_lds or dgrad_bn_backward_recompute or wgrad or bnrelu_on_load or conv3x3_band" -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_deterministic_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_det.log 2>&1 || exit $?
timeout -k 10 200 python tools/conv_bench.py --only dgrad,dgbn --iters 20 > gpurun_out/${tag}_cb_base.log 2>&1 || exit $?
timeout -k 10 200 env RN_TUNE=27=1 python tools/conv_bench.py --only dgbn --iters 20 > gpurun_out/${tag}_cb_xpl.log 2>&1 || exit $?
timeout -k 10 200 env RN_TUNE=21=100 python tools/conv_bench.py --only wgrad --iters 20 > gpurun_out/${tag}_wg_new.log 2>&1 || exit $?
timeout -k 10 200 env RN_TUNE=21=100 RN_LIB_PATH=experiments/librn_base.so RN_LIB_ALLOW_MISMATCH=1 python tools/conv_bench.py --only wgrad --iters 20 > gpurun_out/${tag}_wg_old.log 2>&1 || exit $?
for i in 1 2; do
timeout -k 10 200 env RN_LIB_PATH=experiments/librn_base.so RN_LIB_ALLOW_MISMATCH=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_c2_old$i.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_c2_new$i.log 2>&1 || exit $?
timeout -k 10 200 env RN_TUNE=27=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_c2_xpl$i.log 2>&1 || exit $?
done
