# grouped weight gradient: diagonal blocks spread over four waves (14 = 0) vs on two waves (14 = 2) vs unskipped (1), same box
tools/gpu_steps.sh \
 "300 python -u -m pytest tests/test_kernels_gpu.py -k 'grouped' -x -q --timeout 120 --timeout-method thread > gpurun_out/gw3_kern.log 2>&1" \
 "120 env RN_TUNE=14=0 python tools/conv_bench.py --graph resnext50 --only wgrad --filter conv2 --iters 10 > gpurun_out/gw3_cb_0.log 2>&1" \
 "120 env RN_TUNE=14=2 python tools/conv_bench.py --graph resnext50 --only wgrad --filter conv2 --iters 10 > gpurun_out/gw3_cb_2.log 2>&1" \
 "120 env RN_TUNE=14=1 python tools/conv_bench.py --graph resnext50 --only wgrad --filter conv2 --iters 10 > gpurun_out/gw3_cb_1.log 2>&1" \
 "120 env RN_TUNE=14=0 python tools/conv_bench.py --graph resnext50 --only wgrad --filter conv2 --iters 10 > gpurun_out/gw3_cb_0b.log 2>&1" \
 "120 env RN_TUNE=14=2 python tools/conv_bench.py --graph resnext50 --only wgrad --filter conv2 --iters 10 > gpurun_out/gw3_cb_2b.log 2>&1" \
 "150 env RN_TUNE=14=0 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/gw3_b0.log 2>&1" \
 "150 env RN_TUNE=14=2 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/gw3_b2.log 2>&1" \
 "150 env RN_TUNE=14=0 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/gw3_b0b.log 2>&1" \
 "150 env RN_TUNE=14=2 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/gw3_b2b.log 2>&1"
