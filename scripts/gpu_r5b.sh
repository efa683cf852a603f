# Round-5 session 1: the step parity tests (paired scatter, split MLP list), same-box A/B (the
# round-4 build, the MLP-list build (mid), the working tree x scatter kernels 0 / 4), the scatter's per-level-quarter split
# (timing build), then the other GPU tests and the headline bench line. Usage: bash scripts/gpu_r5b.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${1:-r5b}
timeout -k 10 800 python -u -m pytest tests/test_gpu_step.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_${TAG}_step.log 2>&1 || { tail -40 gpurun_out/tests_${TAG}_step.log; exit 2; }
tail -3 gpurun_out/tests_${TAG}_step.log
for rep in 1 2; do
  LIBS="libnof_prev.so libnof_mid.so" FRAMES=64 SKS=0 ABL_ONLY=full bash scripts/gpu_ab.sh ${TAG}_ab || exit 3
  LIBS=libnof.so FRAMES=64 SKS="0 4" ABL_ONLY=full bash scripts/gpu_ab.sh ${TAG}_ab || exit 3
done
LIBS=libnof_ablate.so FRAMES=64 SKS=0 ABL_ONLY=full,skip_lv0_3,skip_lv4_7,skip_lv8_11,skip_lv12_15,skip_all_levels bash scripts/gpu_ab.sh ${TAG}_split || exit 4
bash scripts/gpu_run.sh $TAG tests=tests/test_gpu_headline.py,tests/test_gpu_optim.py,tests/test_gpu_graph.py,tests/test_gpu_dp.py quick
