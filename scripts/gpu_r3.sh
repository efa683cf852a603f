# Round-3 GPU call: the LDS-transpose layout probe, timing variants of the timing build
# (ABL_ONLY, scripts/ablate.py) at the 64-frame pool, the bench (headline, round protocol),
# then the given GPU tests, the whole gpu suite and smoke(). Usage: bash scripts/gpu_r3.sh TAG test_ids...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 60 ./scripts/tr_probe.bin > gpurun_out/tr_probe_$TAG.json || { cat gpurun_out/tr_probe_$TAG.json; exit 4; }
cat gpurun_out/tr_probe_$TAG.json
LIBS="${LIBS:-libnof_ablate.so}" FRAMES=64 ABL_ONLY="${ABL_ONLY:-full}" bash scripts/gpu_ab.sh $TAG || exit 5
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 3; }
python -c "import json,sys; d=json.load(open('gpurun_out/bench_$TAG.json')); print({k: d[k] for k in ('value','ms_per_step','round_phases_ms_per_step','kernels')})"
timeout -k 10 400 python -u -m pytest "$@" -x -v --timeout 200 --timeout-method thread > gpurun_out/newtests_$TAG.log 2>&1 || { tail -40 gpurun_out/newtests_$TAG.log; exit 1; }
tail -3 gpurun_out/newtests_$TAG.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 2; }
tail -2 gpurun_out/smoke_$TAG.log
