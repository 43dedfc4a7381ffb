#!/bin/bash
# Parameterised GPU recipe (replaces the one-off tools/runs/r0*_*.sh of rounds 1-3).
# usage: tools/runs/run.sh TAG STEP [STEP ...]
# Each STEP is one GPU step with its own time limit (tools/gpu_steps.sh: stops after a fault, abort,
# segfault or timeout; outputs under gpurun_out/TAG_<step>.log):
#   gputest          the full `-m gpu` suite
#   tests:<-k expr>  a subset of the GPU suite selected by a pytest -k expression
#   smoke            __graft_entry__.smoke()
#   bench            the default bench line (C2, with the CPU baselines)
#   c2 | c4 | c5     the C2 / C4 / C5 bench lines without the CPU baselines
#   c2@K=V[,K=V]     the C2 bench line with RN_TUNE overrides (A/B of a tuning key), same for c4@ / c5@
#   c2%VAR=V[,VAR=V] the C2 bench line under environment variables (A/B of an RN_* knob), same for c4% / c5%
#   lib:MODEL        the MODEL bench line with experiments/librn_base.so (RN_LIB_PATH: A/B of two builds)
#   prof[:model][@K=V] rocprofv3 --kernel-trace --stats of a 5-step bench (+ step breakdown, stream use),
#                    optionally with RN_TUNE overrides
#   pmc[:model]      rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE, SQ group) of a 3-step bench
#   layerwise:<-k>   tests/test_step_bf16_gpu.py layer-by-layer checks selected by -k, printed (-s)
tag=$1; shift
model_of() { case "$1" in c4|resnext50) echo resnext50;; c5|resnet50_int8) echo resnet50_int8;; *) echo resnet50;; esac; }
steps=()
for s in "$@"; do
  case "$s" in
    gputest) steps+=("900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_gputest.log 2>&1");;
    tests:*) steps+=("600 python -u -m pytest tests -m gpu -k '${s#tests:}' -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1");;
    layerwise:*) steps+=("600 python -u -m pytest tests/test_step_bf16_gpu.py -k '${s#layerwise:}' -x -v -s --timeout 500 --timeout-method thread > gpurun_out/${tag}_layerwise.log 2>&1");;
    smoke) steps+=("300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${tag}_smoke.log 2>&1");;
    bench) steps+=("300 python bench.py > gpurun_out/${tag}_bench.log 2>&1");;
    c2|c4|c5) steps+=("200 python bench.py --model $(model_of $s) --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_${s}.log 2>&1");;
    c2@*|c4@*|c5@*) m=${s%%@*}; kv=${s#*@}; lab=$(echo "$kv" | tr '=,' '__')
      steps+=("200 env RN_TUNE=$kv python bench.py --model $(model_of $m) --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_${m}_${lab}.log 2>&1");;
    c2%*|c4%*|c5%*) m=${s%%\%*}; kv=${s#*%}; lab=$(echo "$kv" | tr '=,' '__')
      steps+=("200 env $(echo "$kv" | tr ',' ' ') python bench.py --model $(model_of $m) --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_${m}_${lab}.log 2>&1");;
    lib:*) m=${s#lib:}
      steps+=("200 env RN_LIB_PATH=experiments/librn_base.so RN_LIB_ALLOW_MISMATCH=1 python bench.py --model $(model_of $m) --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_${m}_base.log 2>&1");;
    prof|prof:*|prof@*|prof:*@*) spec=${s#prof}; kv=""; [[ "$spec" == *@* ]] && kv=${spec#*@} && spec=${spec%%@*}
      m=$(model_of "${spec#:}"); lab=${m}$( [ -n "$kv" ] && echo "_$(echo "$kv" | tr '=,' '__')" )
      steps+=("300 env RN_TUNE=$kv bash tools/prof_bench.sh ${tag}_${lab} --model $m --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_prof_${lab}.log 2>&1");;
    pmc|pmc:*) m=$(model_of "${s#pmc:}"); steps+=("900 bash tools/pmc_bench.sh ${tag}_${m} --model $m --steps 3 --warmup 1 --no-cpu-baseline --pcie-steps 0 > gpurun_out/${tag}_pmc_${m}.log 2>&1");;
    *) echo "run.sh: unknown step $s" >&2; exit 2;;
  esac
done
tools/gpu_steps.sh "${steps[@]}"
rc=$?
for f in gpurun_out/${tag}_*.log; do
  [ -f "$f" ] || continue
  echo "--- $f"; tail -n 3 "$f" | cut -c1-400
done
for d in gpurun_out/prof_${tag}_*; do
  [ -f "$d/run_kernel_trace.csv" ] || continue
  python tools/step_breakdown.py "$d/run_kernel_trace.csv" > "$d/step_breakdown.txt" 2>&1
  python tools/stream_util.py "$d/run_kernel_trace.csv" > "$d/stream_util.txt" 2>&1
  head -n 25 "$d/step_breakdown.txt"
done
exit $rc
