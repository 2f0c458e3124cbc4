# usage: bash tools/gpu_prof.sh TAG MODEL DEPTH BATCH   (on the GPU box, from the repo root)
# rocprofv3 kernel trace of 10 hipGraph replays + separate FETCH_SIZE / WRITE_SIZE PMC passes
# (eager launches), joined into per-launch tables under gpurun_out/prof_TAG/.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; MODEL=$2; DEPTH=$3; BATCH=$4
D=gpurun_out/prof_$TAG
mkdir -p $D
export TMPDIR=/tmp
A="--model $MODEL --depth $DEPTH --batch $BATCH"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- \
  python3 tools/layer_table.py run $A --fwd 10 --meta $D/meta.json > $D/trace.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- \
  python3 tools/layer_table.py run $A --fwd 3 --eager --meta $D/meta_f.json > $D/fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- \
  python3 tools/layer_table.py run $A --fwd 3 --eager --meta $D/meta_w.json > $D/write.log 2>&1 || exit $?
python3 tools/layer_table.py join $(ls $D/trace/*/run_kernel_trace.csv $D/trace/run_kernel_trace.csv 2>/dev/null | head -1) $D/meta.json $D/layers.json > $D/layers.txt 2>&1 || exit $?
python3 tools/layer_table.py pmc $D/fetch $D/write $D/meta_f.json $D/traffic.json > $D/traffic.txt 2>&1 || exit $?
tail -1 $D/layers.txt; tail -1 $D/traffic.txt
