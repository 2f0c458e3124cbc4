# round-3 evidence: full GPU suite, smoke, benches (R18 b128 default, R50 b256, MobileNet b512),
# R18 b128 per-launch trace + PMC traffic, module-path kernel statistics
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r3ac_tests.log 2>&1 || { tail -40 gpurun_out/r3ac_tests.log; exit 1; }
tail -2 gpurun_out/r3ac_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3ac_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r3ac_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r3ac_bench.json 2> gpurun_out/r3ac_bench.err || exit $?
cut -c1-250 gpurun_out/r3ac_bench.json
timeout -k 10 300 python -u bench.py --depth 50 --batch 256 --no-cpu-baseline --module-path 0 > gpurun_out/r3ac_bench_r50.json 2>> gpurun_out/r3ac_bench.err || exit $?
timeout -k 10 300 python -u bench.py --model mobilenet --batch 512 --no-cpu-baseline --module-path 0 > gpurun_out/r3ac_bench_mbn.json 2>> gpurun_out/r3ac_bench.err || exit $?
bash tools/gpu_prof.sh r18_b128 resnet 18 128 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_module -o run -- python3 tools/module_prof.py --depth 18 --batch 128 > gpurun_out/prof_module/run.log 2>&1 || exit $?
tail -1 gpurun_out/prof_module/run.log
