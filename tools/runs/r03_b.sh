# layerwise parity tests (fp32 small, then the bf16 bench configuration)
mkdir -p gpurun_out
RN_LAYERWISE_OUT=gpurun_out/r03b_layerwise_fp32.json timeout -k 10 400 python -u -m pytest tests/test_step_bf16_gpu.py -k fp32_layerwise -x -v -s --timeout 380 --timeout-method thread > gpurun_out/r03b_lw_fp32.log 2>&1
echo "fp32 rc=$?"
RN_LAYERWISE_OUT=gpurun_out/r03b_layerwise_bf16.json timeout -k 10 500 python -u -m pytest tests/test_step_bf16_gpu.py -k full_size_layerwise -x -v -s --timeout 480 --timeout-method thread > gpurun_out/r03b_lw_bf16.log 2>&1
echo "bf16 rc=$?"
