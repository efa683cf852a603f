set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_all_at.log 2>&1 || { tail -40 gpurun_out/gpu_all_at.log; exit 1; }
tail -1 gpurun_out/gpu_all_at.log
for b in 1; do
timeout -k 10 300 python bench.py --steps 20 --warmup 30 --blocks-per-cu $b --no-cpu-baseline > gpurun_out/bench_at_$b.json 2> gpurun_out/bench_at_$b.err || { tail -20 gpurun_out/bench_at_$b.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_at_$b.json').read().strip().splitlines()[-1]); print($b, d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['loss'], d['tile_records'])"
done
