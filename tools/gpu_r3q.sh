set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r3q_counters.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*\|TCP_[A-Z0-9_]*\|TA_[A-Z0-9_]*" gpurun_out/r3q_counters.txt | sort -u > gpurun_out/r3q_counter_names.txt
wc -l gpurun_out/r3q_counter_names.txt
