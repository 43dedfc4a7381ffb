#!/bin/bash
# C5 A/B: previous library (librn_prev.so, HEAD before the clip-kernel rewrite) vs the current one
set -e
export PYTHONPATH=$PWD/resnet.mxnet_amd:$PWD/tests:$PYTHONPATH
for i in 1 2; do
  for v in prev cur; do
    if [ $v = prev ]; then export RN_LIB_PATH=$PWD/resnet.mxnet_amd/rn/librn_prev.so; else unset RN_LIB_PATH; fi
    timeout -k 10 200 python bench.py --model resnet50_int8 --steps 30 --warmup 5 --no-cpu-baseline \
      --pcie-steps 0 > gpurun_out/r03x_$v.json 2> gpurun_out/r03x_err.txt
    echo "$v $(python3 -c "import json;print(json.loads(open('gpurun_out/r03x_$v.json').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
unset RN_LIB_PATH
timeout -k 10 240 bash tools/prof_bench.sh r03x --model resnet50_int8 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03x_prof.log 2>&1
python3 tools/step_breakdown.py gpurun_out/prof_r03x/run_kernel_trace.csv > gpurun_out/r03x_breakdown.txt
python3 tools/stream_util.py gpurun_out/prof_r03x/run_kernel_trace.csv > gpurun_out/r03x_streams.txt
grep -n "stem_clip" gpurun_out/r03x_breakdown.txt
