set -o pipefail
cd $GRAFT_REPO_ROOT
for b in 2 3; do
timeout -k 10 300 python bench.py --steps 20 --warmup 30 --blocks-per-cu $b --no-cpu-baseline > gpurun_out/bench_as_$b.json 2> gpurun_out/bench_as_$b.err || { tail -20 gpurun_out/bench_as_$b.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_as_$b.json').read().strip().splitlines()[-1]); print($b, d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['loss'])"
done
