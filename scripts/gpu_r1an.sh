set -o pipefail
cd $GRAFT_REPO_ROOT
for w in 5 30 100; do
timeout -k 10 300 python bench.py --steps 20 --warmup $w --no-cpu-baseline > gpurun_out/bench_an_w$w.json 2> gpurun_out/bench_an_w$w.err || { tail -20 gpurun_out/bench_an_w$w.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_an_w$w.json').read().strip().splitlines()[-1]); print($w, d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['loss'])"
done
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/bench_an_s100.json 2> gpurun_out/bench_an_s100.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/bench_an_s100.json').read().strip().splitlines()[-1]); print('s100', d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['loss'])"
