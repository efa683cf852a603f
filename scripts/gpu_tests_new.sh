# Run the given GPU test files/ids first (stop at the first failure), then the whole
# gpu suite, smoke() and one bench line. Usage: bash scripts/gpu_tests_new.sh TAG test_ids...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 400 python -u -m pytest "$@" -x -v --timeout 200 --timeout-method thread > gpurun_out/newtests_$TAG.log 2>&1 || { tail -40 gpurun_out/newtests_$TAG.log; exit 1; }
tail -3 gpurun_out/newtests_$TAG.log
bash scripts/gpu_check.sh $TAG
