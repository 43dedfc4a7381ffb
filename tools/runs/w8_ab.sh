# 8-wave 3-buffer 256x64 tile (rn_set_tuning 4 = 7) vs the 4-wave 2-buffer form: tests, per-layer, bench, C4 bench
tools/gpu_steps.sh \
 "300 python -u -m pytest tests/test_kernels_gpu.py -k 'big_tiles or grouped' -x -q --timeout 120 --timeout-method thread > gpurun_out/w8_kern.log 2>&1" \
 "120 python tools/conv_bench.py --only fwd,dgrad --filter conv2 --iters 10 > gpurun_out/w8_cb_def.log 2>&1" \
 "120 env RN_TUNE=4=7 python tools/conv_bench.py --only fwd,dgrad --filter conv2 --iters 10 > gpurun_out/w8_cb_7.log 2>&1" \
 "120 env RN_TUNE=4=7 python tools/conv_bench.py --graph resnext50 --only fwd,dgrad --filter conv2 --iters 10 > gpurun_out/w8_cbx_7.log 2>&1" \
 "120 python tools/conv_bench.py --graph resnext50 --only fwd,dgrad --filter conv2 --iters 10 > gpurun_out/w8_cbx_def.log 2>&1" \
 "120 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/w8_def.log 2>&1" \
 "120 env RN_TUNE=4=7 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/w8_7.log 2>&1"
