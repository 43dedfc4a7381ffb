#!/bin/bash
# rocprofv3 kernel-trace --stats of a short bench run; summary copied into profiles/<tag>/
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rm -rf gpurun_out/prof_$tag
rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py "$@"
