# grouped weight-gradient diagonal blocks over all four waves (rn_set_tuning 14 = 0 on, 1 off): tests, per-layer, C4 bench A/B, C4 step parity
tools/gpu_steps.sh \
 "300 python -u -m pytest tests/test_kernels_gpu.py -k 'grouped' -x -q --timeout 120 --timeout-method thread > gpurun_out/gw2_kern.log 2>&1" \
 "300 python -u -m pytest tests/test_step_gpu.py tests/test_step_bf16_gpu.py -k resnext -x -q --timeout 200 --timeout-method thread > gpurun_out/gw2_step.log 2>&1" \
 "120 env RN_TUNE=14=0 python tools/conv_bench.py --graph resnext50 --only wgrad --filter conv2 --iters 10 > gpurun_out/gw2_cb_on.log 2>&1" \
 "120 env RN_TUNE=14=1 python tools/conv_bench.py --graph resnext50 --only wgrad --filter conv2 --iters 10 > gpurun_out/gw2_cb_off.log 2>&1" \
 "150 env RN_TUNE=14=0 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/gw2_on.log 2>&1" \
 "150 env RN_TUNE=14=1 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/gw2_off.log 2>&1" \
 "150 env RN_TUNE=14=0 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/gw2_on2.log 2>&1" \
 "150 env RN_TUNE=14=1 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/gw2_off2.log 2>&1"
