# quantizer pass with magic-number rounding: int8 kernel tests, C5 layerwise, bench pair, profile
tools/gpu_steps.sh \
 "300 python -u -m pytest tests/test_int8_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ab_kt.log 2>&1" \
 "600 python -u -m pytest tests/test_step_bf16_gpu.py -x -q -k 'int8' --timeout 500 --timeout-method thread > gpurun_out/r04ab_lw.log 2>&1" \
 "200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04ab_n1.log 2>&1" \
 "200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04ab_n2.log 2>&1" \
 "300 bash tools/prof_bench.sh r04ab --model resnet50_int8 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0"
tail -n2 gpurun_out/r04ab_kt.log; tail -n2 gpurun_out/r04ab_lw.log
for f in n1 n2; do echo -n "$f "; tail -n1 gpurun_out/r04ab_$f.log | grep -o '"ms_per_step": [0-9.]*'; done
python tools/step_breakdown.py gpurun_out/prof_r04ab/run_kernel_trace.csv | grep bnq
