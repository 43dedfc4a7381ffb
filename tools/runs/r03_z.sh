#!/bin/bash
# write-through conv outputs (rn_set_tuning 18): kernel tests with it on, C2 / C4 bench A/B
set -e
export PYTHONPATH=$PWD/resnet.mxnet_amd:$PWD/tests:$PYTHONPATH
RN_TUNE=18=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "bnstats or bnrelu or dgrad_bn or conv_fwd or conv_bwd" > gpurun_out/r03z_tests.log 2>&1
tail -2 gpurun_out/r03z_tests.log
for m in resnet50 resnext50; do
for i in 1 2 3; do
  for v in 0 1; do
    RN_TUNE=18=$v timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline \
      --pcie-steps 0 > gpurun_out/r03z_${m}_$v.json 2> gpurun_out/r03z_err.txt
    echo "$m wt=$v $(python3 -c "import json;print(json.loads(open('gpurun_out/r03z_${m}_$v.json').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
done
