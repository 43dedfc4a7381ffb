# Round 6: dgrad1x1_stream_kernel (rn_set_tuning 27) -- tests, per-layer A/B, C2 pairs (+ the recomputed BN apply).
# usage: bash tools/runs/r06_d1.sh TAG
set -o pipefail
tag=${1:-r06f}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -k "dgrad1x1_stream or dgrad_bn_backward_recompute or bnred" -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || exit $?
timeout -k 10 200 python tools/conv_bench.py --only dgrad,dgbn --iters 20 > gpurun_out/${tag}_cb_new.log 2>&1 || exit $?
timeout -k 10 200 env RN_TUNE=27=2 python tools/conv_bench.py --only dgrad,dgbn --iters 20 > gpurun_out/${tag}_cb_nh1.log 2>&1 || exit $?
timeout -k 10 200 env RN_TUNE=27=1 python tools/conv_bench.py --only dgrad,dgbn --iters 20 > gpurun_out/${tag}_cb_tile.log 2>&1 || exit $?
for i in 1 2; do
timeout -k 10 200 env RN_TUNE=27=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_c2_tile$i.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_c2_new$i.log 2>&1 || exit $?
timeout -k 10 200 env RN_BN_BWD_RECOMPUTE=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_c2_recomp$i.log 2>&1 || exit $?
done
