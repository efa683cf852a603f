set -o pipefail
cd $GRAFT_REPO_ROOT
for v in nr0 nr8 nr12 nr0 nr8 nr12; do
cp bundlesdf_amd/libnof_$v.so bundlesdf_amd/libnof.so
timeout -k 10 300 python bench.py --steps 20 --warmup 30 --no-cpu-baseline > gpurun_out/bench_aw.json 2> gpurun_out/bench_aw.err || { tail -20 gpurun_out/bench_aw.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_aw.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()})"
done
