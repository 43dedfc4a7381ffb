#!/bin/bash
# stem clip gradient, four elements per wave: tests, probe, C5 bench
set -e
export PYTHONPATH=$PWD/resnet.mxnet_amd:$PWD/tests:$PYTHONPATH
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "stem_quant or int8 or quant" > gpurun_out/r03w_tests.log 2>&1
tail -3 gpurun_out/r03w_tests.log
timeout -k 10 120 python tools/probe/stem_clip_probe.py > gpurun_out/r03w_probe.log 2>&1
cat gpurun_out/r03w_probe.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --model resnet50_int8 --steps 30 --warmup 5 --no-cpu-baseline \
    --pcie-steps 0 > gpurun_out/r03w_c5_$i.json 2> gpurun_out/r03w_err.txt
  echo "c5 $(python3 -c "import json;print(json.loads(open('gpurun_out/r03w_c5_$i.json').read().strip().splitlines()[-1])['ms_per_step'])")"
done
