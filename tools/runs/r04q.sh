# int8-codes weight gradients: kernel tests, C5 layerwise (small), then C5 A/B pairs vs RN_QUANT_CODES_WGRAD=0
b() { echo "200 env $1 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04q_$2.log 2>&1"; }
tools/gpu_steps.sh \
 "300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k int8_codes --timeout 120 --timeout-method thread > gpurun_out/r04q_kt.log 2>&1" \
 "400 python -u -m pytest tests/test_step_bf16_gpu.py -x -q -k 'int8_layerwise_small or int8_layerwise_deferred' --timeout 300 --timeout-method thread > gpurun_out/r04q_lw.log 2>&1" \
 "$(b RN_X=0 n1)" "$(b RN_QUANT_CODES_WGRAD=0 o1)" "$(b RN_X=0 n2)" "$(b RN_QUANT_CODES_WGRAD=0 o2)"
tail -n2 gpurun_out/r04q_kt.log; tail -n2 gpurun_out/r04q_lw.log
for f in n1 o1 n2 o2; do echo -n "$f "; tail -n1 gpurun_out/r04q_$f.log | grep -o '"ms_per_step": [0-9.]*'; done
