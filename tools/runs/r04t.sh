# chunked int8 stem weight gradient: C5 layerwise (small, deferred, full size), stem kernel tests, then C5 A/B vs RN_STEM_CHUNKS=1
b() { echo "200 env $1 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04t_$2.log 2>&1"; }
tools/gpu_steps.sh \
 "600 python -u -m pytest tests/test_step_bf16_gpu.py -x -q -k 'int8' --timeout 500 --timeout-method thread > gpurun_out/r04t_lw.log 2>&1" \
 "300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'stem_clip or int8_codes' --timeout 120 --timeout-method thread > gpurun_out/r04t_kt.log 2>&1" \
 "$(b RN_X=0 n1)" "$(b RN_STEM_CHUNKS=1 o1)" "$(b RN_X=0 n2)" "$(b RN_STEM_CHUNKS=1 o2)"
tail -n2 gpurun_out/r04t_lw.log; tail -n2 gpurun_out/r04t_kt.log
for f in n1 o1 n2 o2; do echo -n "$f "; tail -n1 gpurun_out/r04t_$f.log | grep -o '"ms_per_step": [0-9.]*'; done
