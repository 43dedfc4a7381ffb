# quantizer-pair clips + BN reduction in the later dgrad's epilogue: C5 layerwise (small, full), then A/B pairs
b() { echo "200 env $1 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04z_$2.log 2>&1"; }
tools/gpu_steps.sh \
 "600 python -u -m pytest tests/test_step_bf16_gpu.py -x -q -k 'int8' --timeout 500 --timeout-method thread > gpurun_out/r04z_lw.log 2>&1" \
 "$(b RN_X=0 n1)" "$(b RN_QUANT_PAIR_FUSION=0 o1)" "$(b RN_X=0 n2)" "$(b RN_QUANT_PAIR_FUSION=0 o2)"
tail -n2 gpurun_out/r04z_lw.log
for f in n1 o1 n2 o2; do echo -n "$f "; tail -n1 gpurun_out/r04z_$f.log | grep -o '"ms_per_step": [0-9.]*'; done
