#!/bin/bash
# chunked stem BN-backward apply + wgrad: kernel tests, ResNet step tests, C2/C4 bench A/B
set -e
export PYTHONPATH=$PWD/resnet.mxnet_amd:$PWD/tests:$PYTHONPATH
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "bn_relu or stem or step or smoke" > gpurun_out/r03u_tests.log 2>&1
tail -3 gpurun_out/r03u_tests.log
for m in resnet50 resnext50; do
for c in 1 4 2 1 4 2; do
  RN_STEM_CHUNKS=$c timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline \
    --pcie-steps 0 > gpurun_out/r03u_${m}_${c}.json 2> gpurun_out/r03u_err.txt
  echo "$m chunks=$c $(python3 -c "import json;print(json.loads(open('gpurun_out/r03u_${m}_${c}.json').read().strip().splitlines()[-1])['ms_per_step'])")"
done
done
