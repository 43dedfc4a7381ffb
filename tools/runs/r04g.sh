# grouped RED kernels at 3 waves/SIMD; pool-backward BN0 reduction; C2 / C4 / C5 layerwise; A/B; C2 PMC passes
tools/gpu_steps.sh \
 "400 python -u -m pytest tests/test_kernels_gpu.py tests/test_int8_gpu.py -k 'grouped or dgrad_bn_backward_fusion or bnstats or quant or maxpool' -x -q --timeout 300 --timeout-method thread > gpurun_out/r04g_tests.log 2>&1" \
 "600 python -u -m pytest tests/test_step_bf16_gpu.py -k 'resnext50 or int8_layerwise_small or deferred or test_resnet50_bf16_full_size_layerwise or layerwise_small' -x -v -s --timeout 500 --timeout-method thread > gpurun_out/r04g_layerwise.log 2>&1" \
 "200 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04g_c4_a.log 2>&1" \
 "200 env RN_GROUPED_BN_FUSION=0 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04g_c4_b.log 2>&1" \
 "200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04g_c2_a.log 2>&1" \
 "200 env RN_POOL_BN_FUSION=0 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04g_c2_b.log 2>&1" \
 "200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04g_c2_a2.log 2>&1" \
 "200 env RN_POOL_BN_FUSION=0 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04g_c2_b2.log 2>&1" \
 "200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04g_c5.log 2>&1" \
 "900 bash tools/pmc_bench.sh r04g_resnet50 --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04g_pmc.log 2>&1"
tail -n2 gpurun_out/r04g_tests.log; grep -E "passed|failed|Error" gpurun_out/r04g_layerwise.log | tail -3
for f in c4_a c4_b c2_a c2_b c2_a2 c2_b2 c5; do tail -n1 gpurun_out/r04g_$f.log | cut -c1-150; done
tail -n3 gpurun_out/r04g_pmc.log
