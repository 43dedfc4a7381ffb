# grouped weight gradient: resident blocks per CU used to size the M split (rn_set_tuning 2; default 5 for 64x64 tiles)
tools/gpu_steps.sh \
 "120 python tools/conv_bench.py --graph resnext50 --only wgrad --filter conv2 --iters 10 > gpurun_out/gs_5.log 2>&1" \
 "120 env RN_TUNE=2=3 python tools/conv_bench.py --graph resnext50 --only wgrad --filter conv2 --iters 10 > gpurun_out/gs_3.log 2>&1" \
 "120 env RN_TUNE=2=8 python tools/conv_bench.py --graph resnext50 --only wgrad --filter conv2 --iters 10 > gpurun_out/gs_8.log 2>&1" \
 "120 env RN_TUNE=2=12 python tools/conv_bench.py --graph resnext50 --only wgrad --filter conv2 --iters 10 > gpurun_out/gs_12.log 2>&1" \
 "120 python tools/conv_bench.py --graph resnext50 --only wgrad --filter conv2 --iters 10 > gpurun_out/gs_5b.log 2>&1"
