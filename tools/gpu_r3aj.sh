# module-path autotune: its bitwise test, the full suite, the headline drop-in (forced tiles + autotuned),
# the default bench (module_path_images_per_s)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_tiles.py -k module_autotune > gpurun_out/r3aj_at.log 2>&1 || { tail -40 gpurun_out/r3aj_at.log; exit 1; }
tail -1 gpurun_out/r3aj_at.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r3aj_tests.log 2>&1 || { tail -40 gpurun_out/r3aj_tests.log; exit 1; }
tail -1 gpurun_out/r3aj_tests.log
QNN_MODULE_AUTOTUNE=1 timeout -k 10 300 python -u bench_layers.py --only headline r50_l4 > gpurun_out/r3aj_headline.jsonl 2> gpurun_out/r3aj.err || exit $?
timeout -k 10 300 python -u bench_layers.py --only headline r50_l4 --tiles 6 9 26 30 > gpurun_out/r3aj_headline_tiles.jsonl 2>> gpurun_out/r3aj.err || exit $?
python -c "
import json
for f in ['gpurun_out/r3aj_headline.jsonl','gpurun_out/r3aj_headline_tiles.jsonl']:
    for l in open(f):
        d=json.loads(l); print(d['layer'], d['cfg'], d['tile'], d['blocks'], d['conv_us'], d['conv_frac'], d['module_us'])
"
QNN_MODULE_AUTOTUNE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3aj_bench.json 2> gpurun_out/r3aj_bench.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/r3aj_bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['module_path_images_per_s'])"
