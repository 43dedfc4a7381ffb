#!/bin/bash
# (+ the tiled wq_pack_kernel)
# C5 A/B: previous library (librn_prev.so, HEAD before the clip-kernel rewrite) vs the current one
set -e
export PYTHONPATH=$PWD/resnet.mxnet_amd:$PWD/tests:$PYTHONPATH
for i in 1 2 3; do
  for v in prev cur; do
    if [ $v = prev ]; then export RN_LIB_PATH=$PWD/resnet.mxnet_amd/rn/librn_prev.so; else unset RN_LIB_PATH; fi
    timeout -k 10 200 python bench.py --model resnet50_int8 --steps 30 --warmup 5 --no-cpu-baseline \
      --pcie-steps 0 > gpurun_out/r03y_$v.json 2> gpurun_out/r03y_err.txt
    echo "$v $(python3 -c "import json;print(json.loads(open('gpurun_out/r03y_$v.json').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
unset RN_LIB_PATH
timeout -k 10 240 bash tools/prof_bench.sh r03y --model resnet50_int8 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03y_prof.log 2>&1
python3 tools/step_breakdown.py gpurun_out/prof_r03y/run_kernel_trace.csv > gpurun_out/r03y_breakdown.txt
python3 tools/stream_util.py gpurun_out/prof_r03y/run_kernel_trace.csv > gpurun_out/r03y_streams.txt
grep -n "stem_clip" gpurun_out/r03y_breakdown.txt
grep -n "wq_pack\|sgd_mom" gpurun_out/r03y_breakdown.txt
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "weight_quant or int8 or quant" > gpurun_out/r03y_tests.log 2>&1
tail -2 gpurun_out/r03y_tests.log
