# rocprofv3 kernel stats + PMC HBM-traffic passes + per-workload benches (round 1 refresh)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run_wl () {  # name, args
  local nm=$1; shift
  timeout -k 10 240 python3 -u $R/profile_engine.py "$@" --reps 3 > $O/prof_$nm.log 2>&1
  local tiles=$(python3 -c "import json,sys; print(','.join(str(json.loads(l)['cfg']) for l in open('$O/prof_$nm.log') if l.startswith('{') and 'cfg' in l))")
  echo "$nm tiles $tiles"
  QNN_ENGINE_TILES=$tiles timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmcf_$nm -o p -- python3 $R/profile_engine.py "$@" --reps 3 > $O/pmcf_$nm.log 2>&1
  QNN_ENGINE_TILES=$tiles timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmcw_$nm -o p -- python3 $R/profile_engine.py "$@" --reps 3 > $O/pmcw_$nm.log 2>&1
  QNN_ENGINE_TILES=$tiles timeout -k 10 200 python3 -u $R/profile_engine.py "$@" --reps 3 > $O/prof2_$nm.log 2>&1
  python3 $R/tools/traffic.py $O/pmcf_$nm $O/pmcw_$nm $O/prof2_$nm.log $O/traffic_$nm.json
}
run_wl resnet18_b128 --depth 18 --batch 128
run_wl resnet50_b256 --depth 50 --batch 256
run_wl mobilenet_b512 --model mobilenet --batch 512
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp_r18 -o rp -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --module-path 0 > $O/rp_r18.log 2>&1
timeout -k 10 300 python3 -u $R/bench.py --depth 50 --batch 256 --steps 10 --warmup 3 --cpu-batch 2 --cpu-iters 3 > $O/bench_r50.log 2>&1
timeout -k 10 300 python3 -u $R/bench.py --model mobilenet --batch 512 --steps 10 --warmup 3 --cpu-batch 4 --cpu-iters 3 > $O/bench_mbn.log 2>&1
