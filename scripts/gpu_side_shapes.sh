# Final-build side shapes: BASELINE config 5 (global refine) per-GPU step and the 8-frame per-rank batch of N = 8.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload global_refine > gpurun_out/bench_global_refine_r6w.json 2> gpurun_out/bench_gr_r6w.err || { tail -20 gpurun_out/bench_gr_r6w.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/bench_global_refine_r6w.json')); print(d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()})"
timeout -k 10 300 python bench.py --pool-frames 8 --no-extras --no-cpu-baseline > gpurun_out/bench_8frames_per_rank_r6w.json 2> gpurun_out/bench_8f_r6w.err || { tail -20 gpurun_out/bench_8f_r6w.err; exit 4; }
python -c "import json; d=json.load(open('gpurun_out/bench_8frames_per_rank_r6w.json')); print(d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()})"
