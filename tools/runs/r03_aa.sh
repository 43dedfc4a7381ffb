#!/bin/bash
# BN merge / finalize kernels with their loads hoisted: BN tests, C2 / C4 A/B vs the previous library
set -e
export PYTHONPATH=$PWD/resnet.mxnet_amd:$PWD/tests:$PYTHONPATH
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "bn or bnstats or step" > gpurun_out/r03aa_tests.log 2>&1
tail -2 gpurun_out/r03aa_tests.log
for m in resnet50 resnext50; do
for i in 1 2 3; do
  for v in prev cur; do
    if [ $v = prev ]; then export RN_LIB_PATH=$PWD/resnet.mxnet_amd/rn/librn_prev.so; else unset RN_LIB_PATH; fi
    timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline \
      --pcie-steps 0 > gpurun_out/r03aa_${m}_$v.json 2> gpurun_out/r03aa_err.txt
    echo "$m $v $(python3 -c "import json;print(json.loads(open('gpurun_out/r03aa_${m}_$v.json').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
done
unset RN_LIB_PATH
timeout -k 10 240 bash tools/prof_bench.sh r03aa --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r03aa_prof.log 2>&1
python3 tools/step_breakdown.py gpurun_out/prof_r03aa/run_kernel_trace.csv > gpurun_out/r03aa_breakdown.txt
grep -n "finalize\|merge" gpurun_out/r03aa_breakdown.txt
