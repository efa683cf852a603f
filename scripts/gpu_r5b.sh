set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py -m gpu -x -v --timeout 300 --timeout-method thread -k "pair or headline or amp_matches" > gpurun_out/tests_r5b_pair.log 2>&1 || { tail -40 gpurun_out/tests_r5b_pair.log; exit 2; }
tail -3 gpurun_out/tests_r5b_pair.log
LIBS=libnof.so FRAMES=64 SKS="0 4 0 4" ABL_ONLY=full bash scripts/gpu_ab.sh r5b_pair || exit 3
LIBS=libnof_ablate.so FRAMES=64 SKS=0 ABL_ONLY=full,skip_lv0_3,skip_lv4_7,skip_lv8_11,skip_lv12_15,skip_all_levels bash scripts/gpu_ab.sh r5b_split || exit 4
bash scripts/gpu_run.sh r5b tests=tests/test_gpu_headline.py,tests/test_gpu_optim.py,tests/test_gpu_graph.py,tests/test_gpu_dp.py quick
