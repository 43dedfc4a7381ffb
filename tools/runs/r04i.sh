# weight-gradient split grids sized for a fraction of the chip (rn_set_tuning 21): C2 / C4 / C5 A/B
tools/gpu_steps.sh \
 "300 python -u -m pytest tests/test_int8_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04i_int8.log 2>&1" \
 "300 python -u -m pytest tests/test_kernels_gpu.py -k 'stem' -x -q --timeout 300 --timeout-method thread > gpurun_out/r04i_stem.log 2>&1" \
 "400 python -u -m pytest tests/test_step_bf16_gpu.py -k 'int8_layerwise_small or int8_full_size' -x -q --timeout 300 --timeout-method thread > gpurun_out/r04i_lw.log 2>&1" \
 "300 env RN_TUNE=21=50 python -u -m pytest tests/test_kernels_gpu.py -k 'wgrad or image_bands or stream_1x1' -x -q --timeout 300 --timeout-method thread > gpurun_out/r04i_tests.log 2>&1" \
 "200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c2_100.log 2>&1" \
 "200 env RN_TUNE=21=50 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c2_50.log 2>&1" \
 "200 env RN_TUNE=21=25 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c2_25.log 2>&1" \
 "200 env RN_TUNE=21=75 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c2_75.log 2>&1" \
 "200 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c2_100b.log 2>&1" \
 "200 env RN_TUNE=21=50 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c2_50b.log 2>&1" \
 "200 env RN_TUNE=21=25 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c2_25b.log 2>&1" \
 "200 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c4_100.log 2>&1" \
 "200 env RN_TUNE=21=50 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c4_50.log 2>&1" \
 "200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c5_100.log 2>&1" \
 "200 env RN_TUNE=21=50 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c5_50.log 2>&1" \
 "200 env RN_TUNE=22=1 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c5_div.log 2>&1" \
 "200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c5_100b.log 2>&1" \
 "200 env RN_TUNE=22=1 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c5_divb.log 2>&1" \
 "200 env RN_STEM_CLIP_MASK=0 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c5_gather.log 2>&1" \
 "200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c5_100c.log 2>&1" \
 "200 env RN_STEM_CLIP_MASK=0 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04i_c5_gatherb.log 2>&1"
tail -n2 gpurun_out/r04i_int8.log; tail -n2 gpurun_out/r04i_stem.log; tail -n2 gpurun_out/r04i_lw.log; tail -n2 gpurun_out/r04i_tests.log
for f in c2_100 c2_50 c2_25 c2_75 c2_100b c2_50b c2_25b c4_100 c4_50 c5_100 c5_50 c5_div c5_100b c5_divb c5_gather c5_100c c5_gatherb; do echo -n "$f "; tail -n1 gpurun_out/r04i_$f.log | grep -o '"ms_per_step": [0-9.]*'; done
