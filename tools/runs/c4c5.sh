# BASELINE C4 (ResNeXt-50 32x4d) and C5 (resnet_int8) on one GPU: bench lines + a one-stream kernel trace of C4
tools/gpu_steps.sh \
 "200 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/c4_bench.log 2>&1" \
 "200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/c5_bench.log 2>&1" \
 "240 env RN_WGRAD_STREAM=0 bash tools/prof_bench.sh c41s --model resnext50 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/c41s_prof.log 2>&1"
