# grouped weight gradient at 8 blocks per CU (new default) vs 5 (RN_TUNE=2=5, forces every wgrad_kernel layer): tests, C4 bench pairs
tools/gpu_steps.sh \
 "300 python -u -m pytest tests/test_kernels_gpu.py -k 'grouped' -x -q --timeout 120 --timeout-method thread > gpurun_out/gs2_kern.log 2>&1" \
 "300 python -u -m pytest tests/test_step_gpu.py tests/test_step_bf16_gpu.py -k resnext -x -q --timeout 200 --timeout-method thread > gpurun_out/gs2_step.log 2>&1" \
 "120 python tools/conv_bench.py --graph resnext50 --only wgrad --iters 10 > gpurun_out/gs2_cb_new.log 2>&1" \
 "120 env RN_TUNE=2=5 python tools/conv_bench.py --graph resnext50 --only wgrad --iters 10 > gpurun_out/gs2_cb_5.log 2>&1" \
 "150 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/gs2_new.log 2>&1" \
 "150 env RN_TUNE=14=0 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/gs2_new2.log 2>&1" \
 "150 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/gs2_r50.log 2>&1"
