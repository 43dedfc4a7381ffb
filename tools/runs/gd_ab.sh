# grouped zero-block MFMA skip (rn_set_tuning 13 = 0 on, 1 off): tests, per-layer, C4 bench A/B, C4 step parity
tools/gpu_steps.sh \
 "300 python -u -m pytest tests/test_kernels_gpu.py -k 'grouped' -x -q --timeout 120 --timeout-method thread > gpurun_out/gd_kern.log 2>&1" \
 "300 env RN_TUNE=13=0 python -u -m pytest tests/test_step_gpu.py tests/test_step_bf16_gpu.py -k resnext -x -q --timeout 200 --timeout-method thread > gpurun_out/gd_step.log 2>&1" \
 "120 env RN_TUNE=13=0 python tools/conv_bench.py --graph resnext50 --only fwd,dgrad --filter conv2 --iters 10 > gpurun_out/gd_cb_on.log 2>&1" \
 "120 env RN_TUNE=13=1 python tools/conv_bench.py --graph resnext50 --only fwd,dgrad --filter conv2 --iters 10 > gpurun_out/gd_cb_off.log 2>&1" \
 "150 env RN_TUNE=13=0 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/gd_on.log 2>&1" \
 "150 env RN_TUNE=13=1 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/gd_off.log 2>&1" \
 "150 env RN_TUNE=13=0 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/gd_on2.log 2>&1"
