#!/bin/bash
# SQ/LDS counters for one conv layer's kernels (tools/conv_bench.py), one counter group per pass.
# usage: tools/pmc_conv.sh <tag> <conv_bench args...>
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
groups=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES"
        "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT")
i=0
for g in "${groups[@]}"; do
  rm -rf gpurun_out/pmcc_${tag}_$i
  timeout -k 10 300 rocprofv3 --pmc $g --kernel-trace -d gpurun_out/pmcc_${tag}_$i -o run --output-format csv -- python3 tools/conv_bench.py "$@" || exit $?
  i=$((i+1))
done
