# round 4 first run: the ADVICE / verdict fixes, the new C4 / C5 layerwise checks and the image-band
# weight gradient on the GPU, then C2 (band wgrad on / off), C4, C5 bench lines
tools/gpu_steps.sh \
 "400 python -u -m pytest tests/test_int8_gpu.py tests/test_bench_launch.py tests/test_kernels_gpu.py -k 'weight_quant_pack or gpus2 or grouped_conv_direct or zero_block or image_bands or stream_1x1 or grouped_image_bands or big_tiles' -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a_tests.log 2>&1" \
 "400 python -u -m pytest tests/test_step_bf16_gpu.py -k 'layerwise_small' -v -s --timeout 300 --timeout-method thread > gpurun_out/r04a_lw_small.log 2>&1" \
 "200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04a_c2.log 2>&1" \
 "200 env RN_TUNE=19=1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04a_c2_noband.log 2>&1" \
 "200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04a_c2b.log 2>&1" \
 "200 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04a_c4.log 2>&1" \
 "200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04a_c5.log 2>&1"
tail -n3 gpurun_out/r04a_tests.log; tail -n5 gpurun_out/r04a_lw_small.log; for f in c2 c2_noband c2b c4 c5; do tail -n1 gpurun_out/r04a_$f.log | cut -c1-200; done
