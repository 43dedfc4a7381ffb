#!/bin/bash
# PMC passes over a short bench run, one counter group per pass (gfx950: FETCH_SIZE and WRITE_SIZE
# cannot share a pass; SQ group <= 8 SQ + 2 GRBM counters). Output: gpurun_out/pmc_<tag>_{fetch,write,sq}/
# usage: tools/pmc_bench.sh <tag> <bench.py args...>
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() {  # $1 = pass name, rest = counters
  local name=$1; shift
  rm -rf gpurun_out/pmc_${tag}_$name
  timeout -k 10 400 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/pmc_${tag}_$name -o run \
    --output-format csv -- python3 bench.py $BENCH_ARGS || exit $?
}
BENCH_ARGS="$*"
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE
