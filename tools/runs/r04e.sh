# grouped BN fusions (direct-kernel / block-diagonal-tile BN-backward reduction, tile statistics):
# kernel tests, C4 layerwise, C4 A/B (fusion off, stride-2 GD dgrad tile), conv_bench dgrad
tools/gpu_steps.sh \
 "400 python -u -m pytest tests/test_kernels_gpu.py -k 'grouped or dgrad_bn_backward_fusion or bnstats' -x -q --timeout 300 --timeout-method thread > gpurun_out/r04e_tests.log 2>&1" \
 "500 python -u -m pytest tests/test_step_bf16_gpu.py -k 'resnext50' -x -v -s --timeout 450 --timeout-method thread > gpurun_out/r04e_layerwise.log 2>&1" \
 "200 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04e_c4_a.log 2>&1" \
 "200 env RN_GROUPED_BN_FUSION=0 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04e_c4_b.log 2>&1" \
 "200 env RN_TUNE=13=2 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04e_c4_c.log 2>&1" \
 "200 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04e_c4_a2.log 2>&1" \
 "200 env RN_GROUPED_BN_FUSION=0 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04e_c4_b2.log 2>&1" \
 "200 python tools/conv_bench.py --graph resnext50 --only dgrad > gpurun_out/r04e_cb_d.log 2>&1" \
 "200 env RN_TUNE=13=2 python tools/conv_bench.py --graph resnext50 --only dgrad > gpurun_out/r04e_cb_d2.log 2>&1"
tail -n2 gpurun_out/r04e_tests.log; grep -E "passed|failed|Error" gpurun_out/r04e_layerwise.log | tail -3
for f in c4_a c4_b c4_c c4_a2 c4_b2; do tail -n1 gpurun_out/r04e_$f.log | cut -c1-150; done
tail -n1 gpurun_out/r04e_cb_d.log; tail -n1 gpurun_out/r04e_cb_d2.log
