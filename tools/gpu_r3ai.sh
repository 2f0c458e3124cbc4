# headline drop-in (fp32 NCHW boundary): every candidate tile configuration forced
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench_layers.py --only headline r50_l4 --tiles 0 6 9 12 26 28 30 34 > gpurun_out/r3ai_headline_tiles.jsonl 2> gpurun_out/r3ai.err || { tail -20 gpurun_out/r3ai.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r3ai_headline_tiles.jsonl'):
    d=json.loads(l); print(d['layer'], d['cfg'], d['tile'], d['blocks'], d['conv_us'], d['conv_frac'], d['module_us'])
"
