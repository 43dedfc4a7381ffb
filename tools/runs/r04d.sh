# stage-1-only band / act2 fusion: kernel tests, C2 layerwise, C2 A/B of the act2 fusion (pairs), C4, C5
tools/gpu_steps.sh \
 "400 python -u -m pytest tests/test_kernels_gpu.py -k 'image_bands or stream_1x1 or bnrelu_on_load or big_tiles' -x -q --timeout 300 --timeout-method thread > gpurun_out/r04d_tests.log 2>&1" \
 "400 python -u -m pytest tests/test_step_bf16_gpu.py -k 'test_resnet50_bf16_full_size_layerwise or step_gradients' -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04d_layerwise.log 2>&1" \
 "200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04d_c2_a.log 2>&1" \
 "200 env RN_BN_APPLY_FUSION_3X3=0 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04d_c2_b.log 2>&1" \
 "200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04d_c2_a2.log 2>&1" \
 "200 env RN_BN_APPLY_FUSION_3X3=0 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04d_c2_b2.log 2>&1" \
 "200 env RN_TUNE=19=1 RN_BN_APPLY_FUSION_3X3=0 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04d_c2_c.log 2>&1" \
 "200 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04d_c4.log 2>&1" \
 "200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04d_c5.log 2>&1" \
 "200 python tools/conv_bench.py --only fwd,dgrad > gpurun_out/r04d_cb_fd.log 2>&1" \
 "300 bash tools/prof_bench.sh r04d_c5 --model resnet50_int8 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04d_prof_c5.log 2>&1" \
 "300 bash tools/prof_bench.sh r04d_c4 --model resnext50 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04d_prof_c4.log 2>&1"
tail -n2 gpurun_out/r04d_tests.log; grep -E "passed|failed" gpurun_out/r04d_layerwise.log | tail -2
for f in c2_a c2_b c2_a2 c2_b2 c2_c c4 c5; do tail -n1 gpurun_out/r04d_$f.log | cut -c1-150; done
tail -n1 gpurun_out/r04d_cb_fd.log
for d in gpurun_out/prof_r04d_c5 gpurun_out/prof_r04d_c4; do python tools/step_breakdown.py $d/run_kernel_trace.csv > $d/step_breakdown.txt; python tools/stream_util.py $d/run_kernel_trace.csv > $d/stream_util.txt; head -25 $d/step_breakdown.txt; done
