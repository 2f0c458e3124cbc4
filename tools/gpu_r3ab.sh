# residual code chain length vs fp32 checkpoints: bench at QNN_ENGINE_MAX_LINKS = 0..4 (R18 b128, R50 b256)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for L in 0 1 2 3 4; do
QNN_ENGINE_MAX_LINKS=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --module-path 0 > gpurun_out/r3ab_r18_L$L.json 2>> gpurun_out/r3ab.err || exit $?
echo "r18 L=$L $(python -c "import json;d=json.load(open('gpurun_out/r3ab_r18_L$L.json'));print(d['ms_per_step'], d['value'])")"
done
for L in 0 1 2 3 4; do
QNN_ENGINE_MAX_LINKS=$L timeout -k 10 300 python -u bench.py --depth 50 --batch 256 --no-cpu-baseline --module-path 0 > gpurun_out/r3ab_r50_L$L.json 2>> gpurun_out/r3ab.err || exit $?
echo "r50 L=$L $(python -c "import json;d=json.load(open('gpurun_out/r3ab_r50_L$L.json'));print(d['ms_per_step'], d['value'])")"
done
