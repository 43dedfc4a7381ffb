# int8-codes weight gradients: the kernel tests, C5 layerwise small + deferred, then full size
tools/gpu_steps.sh \
 "300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k int8_codes --timeout 120 --timeout-method thread > gpurun_out/r04r_kt.log 2>&1" \
 "400 python -u -m pytest tests/test_step_bf16_gpu.py -x -q -k 'int8_layerwise' --timeout 400 --timeout-method thread > gpurun_out/r04r_lw.log 2>&1"
tail -n2 gpurun_out/r04r_kt.log; tail -n2 gpurun_out/r04r_lw.log
