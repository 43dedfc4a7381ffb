#!/bin/bash
# batched grouped repacks: kernel tests, ResNeXt steps, C4 bench A/B
set -e
export PYTHONPATH=$PWD/resnet.mxnet_amd:$PWD/tests:$PYTHONPATH
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "weight_pack_multi or grouped or resnext" > gpurun_out/r03t_tests.log 2>&1
tail -3 gpurun_out/r03t_tests.log
for b in 0 1 0 1; do
  RN_GPACK_BATCH=$b timeout -k 10 200 python bench.py --model resnext50 --steps 30 --warmup 5 --no-cpu-baseline \
    --pcie-steps 0 > gpurun_out/r03t_b$b.json 2> gpurun_out/r03t_b$b.err
  echo "batch=$b $(python3 -c "import json;print(json.loads(open('gpurun_out/r03t_b$b.json').read().strip().splitlines()[-1])['ms_per_step'])")"
done
