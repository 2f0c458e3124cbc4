# One parametrised GPU-box runner (replaces the per-experiment scripts of earlier rounds).
# usage (on the box, from the repo root):  bash tools/gpu.sh TAG STEP [STEP ...]
# steps:
#   tests              the whole -m gpu suite
#   test:PATH[::K]     one test file / node
#   pyt:ARGS           pytest -m gpu with ARGS (comma-separated; '+' inside an argument is a space,
#                      e.g. pyt:tests/test_gpu_tiles.py,-k,45+or+46)
#   smoke              __graft_entry__.smoke()
#   bench[:ARGS]       python bench.py ARGS  (ARGS: comma-separated, e.g. bench:--depth,50,--batch,256)
#   prof:MODEL:DEPTH:BATCH   tools/gpu_prof.sh (kernel trace of 10 graph replays + PMC traffic)
#   benchprof[:ARGS]   rocprofv3 --kernel-trace --stats of the bench command itself
#   tracecheck[:ARGS]  tools/trace_check.py on that trace and bench line (same ARGS)
#   pmc:MODEL:DEPTH:BATCH:C1,C2,..  one rocprofv3 --pmc pass (eager launches) + tools/pmc_table.py
#   py:SCRIPT[:ARGS]   python SCRIPT ARGS (comma-separated)
# Every step runs under its own timeout; the first failing step ends the run.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
for S in "$@"; do
  KIND=${S%%:*}; ARG=${S#*:}; [ "$ARG" = "$S" ] && ARG=""
  ARGS=${ARG//,/ }
  echo "=== $S $(date +%T)"
  case $KIND in
    tests) timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
           rc=$?; tail -3 $O/tests.log ;;
    test) N=$(echo "$ARG" | tr '/:' '__')
          timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu $ARG > $O/test_$N.log 2>&1
          rc=$?; tail -3 $O/test_$N.log ;;
    pyt) IFS=, read -r -a PA <<< "$ARG"; PA=("${PA[@]//+/ }")
         timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "${PA[@]}" > $O/pyt.log 2>&1
         rc=$?; tail -5 $O/pyt.log ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
           rc=$?; tail -1 $O/smoke.log ;;
    bench) N=$(echo "$ARGS" | tr -d ' -' | head -c 40)
           timeout -k 10 400 python -u bench.py $ARGS > $O/bench_$N.json 2> $O/bench_$N.err
           rc=$?; cut -c1-400 $O/bench_$N.json; [ $rc -ne 0 ] && tail -20 $O/bench_$N.err ;;
    benchprof) N=$(echo "$ARGS" | tr -d ' -' | head -c 40)
           timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/benchprof_$N -o run -- \
             python3 bench.py --no-cpu-baseline --module-path 0 $ARGS > $O/benchprof_$N.json 2> $O/benchprof_$N.err
           rc=$?; cut -c1-300 $O/benchprof_$N.json ;;
    prof) IFS=: read -r M D B <<< "$ARG"
          bash tools/gpu_prof.sh ${TAG}_${M}${D}_b$B $M $D $B; rc=$? ;;
    pmc) IFS=: read -r M D B CN <<< "$ARG"; CN=${CN//,/ }
         P=$O/pmc_${M}${D}_b$B; mkdir -p $P
         timeout -s KILL 300 rocprofv3 --pmc $CN --output-format csv -d $P/raw -o run -- \
           python3 tools/layer_table.py run --model $M --depth $D --batch $B --fwd 2 --eager --meta $P/meta.json > $P/run.log 2>&1
         rc=$?; [ $rc -eq 0 ] && python3 tools/pmc_table.py $P/meta.json $P/raw --json $P/pmc.json > $P/pmc.txt 2>&1; rc=$?
         cat $P/pmc.txt | head -70 ;;
    tracecheck) N=$(echo "$ARGS" | tr -d ' -' | head -c 40)
           T=$(ls $O/benchprof_$N/*/run_kernel_trace.csv $O/benchprof_$N/run_kernel_trace.csv 2>/dev/null | head -1)
           python3 tools/trace_check.py $T $O/benchprof_$N.json $O/tracecheck_$N.json; rc=$? ;;
    py) SCR=${ARG%%:*}; PA=${ARG#*:}; [ "$PA" = "$ARG" ] && PA=""; PA=${PA//,/ }
        N=$(basename $SCR .py)
        timeout -k 10 600 python -u $SCR $PA > $O/$N.out 2> $O/$N.err
        rc=$?; tail -30 $O/$N.out; [ $rc -ne 0 ] && tail -20 $O/$N.err ;;
    *) echo "unknown step $S"; rc=2 ;;
  esac
  echo "=== $S rc=$rc $(date +%T)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
