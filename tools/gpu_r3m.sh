set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_stem_pool.py tests/test_gpu_parity.py > gpurun_out/r3m_stem.log 2>&1
rc=$?; tail -3 gpurun_out/r3m_stem.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/engine_sweep.py --depth 18 --batch 128 --json gpurun_out/r3m_sweep_r18.json > gpurun_out/r3m_sweep_r18.txt 2>&1 || exit $?
grep -v amdgpu gpurun_out/r3m_sweep_r18.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3m_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3m_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['engine'])"
