#!/bin/bash
# HBM traffic counters for a short bench run, one counter group per pass (gfx950: FETCH_SIZE and
# WRITE_SIZE cannot share a pass). Output: gpurun_out/pmc_<tag>_{fetch,write}/
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for c in FETCH_SIZE WRITE_SIZE; do
  low=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  rm -rf gpurun_out/pmc_${tag}_$low
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/pmc_${tag}_$low -o run --output-format csv -- python3 bench.py "$@" || exit $?
done
