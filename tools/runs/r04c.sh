# band-kernel pipelining + act2 BN+ReLU on load: kernel tests, C2 layerwise, isolated wgrad timings
# (band kernels on / off), C2 bench A/B of the 3x3 BN+ReLU fusion
tools/gpu_steps.sh \
 "400 python -u -m pytest tests/test_kernels_gpu.py -k 'image_bands or stream_1x1 or bnrelu_on_load or big_tiles or bnstats or int8 or conv_fwd or conv_bwd' -x -q --timeout 300 --timeout-method thread > gpurun_out/r04c_tests.log 2>&1" \
 "400 python -u -m pytest tests/test_step_bf16_gpu.py -k 'test_resnet50_bf16_full_size_layerwise or test_resnet50_fp32_layerwise or step_gradients' -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04c_layerwise.log 2>&1" \
 "200 python tools/conv_bench.py --only wgrad > gpurun_out/r04c_cb_on.log 2>&1" \
 "200 env RN_TUNE=19=1 python tools/conv_bench.py --only wgrad > gpurun_out/r04c_cb_off.log 2>&1" \
 "200 python tools/conv_bench.py --graph resnext50 --only wgrad > gpurun_out/r04c_cb4_on.log 2>&1" \
 "200 env RN_TUNE=19=1 python tools/conv_bench.py --graph resnext50 --only wgrad > gpurun_out/r04c_cb4_off.log 2>&1" \
 "200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04c_c2_a.log 2>&1" \
 "200 env RN_BN_APPLY_FUSION_3X3=0 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04c_c2_b.log 2>&1" \
 "200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04c_c2_a2.log 2>&1" \
 "200 env RN_BN_APPLY_FUSION_3X3=0 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04c_c2_b2.log 2>&1" \
 "200 env RN_TUNE=19=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04c_c2_c.log 2>&1" \
 "200 env RN_TUNE=20=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04c_c2_p.log 2>&1" \
 "200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04c_c2_a3.log 2>&1" \
 "200 env RN_TUNE=20=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04c_c2_p2.log 2>&1" \
 "200 env RN_TUNE=20=2 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04c_c2_s.log 2>&1" \
 "200 env RN_TUNE=20=2 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04c_c2_s2.log 2>&1"
tail -n3 gpurun_out/r04c_tests.log; grep -E "passed|failed" gpurun_out/r04c_layerwise.log | tail -3
for f in cb_on cb_off cb4_on cb4_off; do tail -n1 gpurun_out/r04c_$f.log; done
for f in c2_a c2_b c2_a2 c2_b2 c2_c c2_p c2_a3 c2_p2 c2_s c2_s2; do tail -n1 gpurun_out/r04c_$f.log | cut -c1-150; done
