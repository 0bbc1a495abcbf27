#!/bin/bash
# The one GPU-box runner: a named sequence of steps, each under its own time
# limit, stopping at the first failure (no retries).  Output under
# gpurun_out/<TAG>/.
#
# Usage (on the box):  bash tools/gpu.sh TAG STEP [STEP ...]
#   suite            whole `-m gpu` test suite (pytest_gpu.log)
#   pytest:ARGS      pytest -m gpu with ARGS ('+' stands for a space), e.g.
#                    pytest:tests/test_gpu_steady.py+-k+step64
#   smoke            __graft_entry__.smoke()
#   bench[:ARGS]     python bench.py ARGS (bench.log; the driver's command
#                    when ARGS is empty)
#   configs          python bench.py --configs (cfg.log)
#   trace[:ARGS]     rocprofv3 --kernel-trace --stats of bench.py ARGS (trace/)
#   pmc              FETCH_SIZE and WRITE_SIZE passes of the headline leg (pmc_*/)
#   ab64             d = 64 step launch time, release library vs every
#                    lib/var_*/ variant (tools/build_variants.sh), twice
#   ab:SCRIPT+ARGS   the same A/B for any python tool script
#   py:SCRIPT+ARGS   one python tool script
#   rocpy:NAME:SCRIPT+ARGS   rocprofv3 --kernel-trace --stats of a tool script (NAME/)
#   pmcpy:NAME:SCRIPT+ARGS   FETCH_SIZE / WRITE_SIZE passes of a tool script (NAME/pmc_*/;
#                    tools/pooled_pmc_summary.py gpurun_out/TAG/NAME)
# Summaries: tools/prof_summary.py TAG --src gpurun_out/TAG after `trace pmc`
# (the step kernel's trace + FETCH/WRITE -> profiles/TAG_step_kernel.json).
# (The per-round gpu_r*.sh / gpu_ab*.sh scripts of rounds 1-5 are folded in here.)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
( while sleep 60; do echo "[$(date +%T)] $(ls -t $O 2>/dev/null | head -1): $(tail -n 1 $O/$(ls -t $O | head -1) 2>/dev/null | cut -c1-100)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT

NPY=0
run() {  # run LIMIT LOG cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$log 2>&1
  local rc=$?
  echo "[$log] rc=$rc"
  grep -v amdgpu.ids $O/$log | tail -n 3 | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}

for step in "$@"; do
  arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  args=${arg//+/ }
  case ${step%%:*} in
    suite) run 1200 pytest_gpu.log python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread --durations=15 ;;
    pytest) run 900 pytest_part.log python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread $args ;;
    smoke) run 300 smoke.log python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    bench) run 400 bench.log python3 bench.py $args ;;
    configs) run 600 cfg.log python3 bench.py --configs ;;
    trace) run 600 trace.log rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py $args ;;
    pmc)
      for C in FETCH_SIZE WRITE_SIZE; do
        run 300 pmc_$C.log rocprofv3 --pmc $C -d $O/pmc_$C -o pmc --output-format csv -- \
          python3 bench.py --steps 20 --warmup 2 --no-extra --no-fused
      done ;;
    ab64|ab)
      cmd="tools/s64_sweep.py 65536"; [ -n "$args" ] && cmd=$args
      for rep in 1 2; do
        for lib in release adaptive-mcmc_amd/lib/var_*/libamh.so; do
          [ -e "$lib" ] || [ $lib = release ] || continue
          if [ $lib = release ]; then n=release; else n=$(basename $(dirname $lib)); fi
          if [ $n = release ]; then
            timeout -k 10 180 python3 $cmd > $O/ab_${n}_$rep.txt 2>&1
          else
            AMH_LIB_PATH=$lib timeout -k 10 180 python3 $cmd > $O/ab_${n}_$rep.txt 2>&1
          fi
          rc=$?; echo "$n: $(grep -v amdgpu.ids $O/ab_${n}_$rep.txt | tail -1)"; [ $rc -eq 0 ] || exit $rc
        done
      done ;;
    py) NPY=$((NPY + 1)); run 600 py${NPY}_$(basename ${args%% *} .py).log python3 -u $args ;;
    rocpy)
      name=${arg%%:*}; rest=${arg#*:}; rest=${rest//+/ }
      run 600 $name.log rocprofv3 --kernel-trace --stats -d $O/$name -o run --output-format csv -- python3 $rest ;;
    pmcpy)
      name=${arg%%:*}; rest=${arg#*:}; rest=${rest//+/ }
      for C in FETCH_SIZE WRITE_SIZE; do
        mkdir -p $O/$name
        run 300 ${name}_pmc_$C.log rocprofv3 --pmc $C -d $O/$name/pmc_$C -o pmc --output-format csv -- python3 $rest
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0
