# Round-4: pose tests + rocprof kernel stats of the headline bench and of the 2048-ray step
# (quick: kernel-trace only). Usage: bash scripts/gpu_r4p.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1
timeout -k 10 300 python -u -m pytest tests/test_gpu_pose.py tests/test_gpu_step.py -k "pose or reference_train_loop" -x -q --timeout 200 --timeout-method thread > gpurun_out/newtests_$TAG.log 2>&1 || { tail -30 gpurun_out/newtests_$TAG.log; exit 1; }
tail -2 gpurun_out/newtests_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python $R/bench.py --warmup 20 --no-cpu-baseline --no-extras > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 3; }
find $R/gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $R/gpurun_out/kernel_stats_$TAG.csv
bash $R/scripts/gpu_small_prof.sh $TAG > $R/gpurun_out/sprof_top_$TAG.txt 2>&1 || { tail -20 $R/gpurun_out/sprof_top_$TAG.txt; exit 4; }
cp $R/gpurun_out/sprof_$TAG/run_kernel_stats.csv $R/gpurun_out/kernel_stats_parity_$TAG.csv
rm -rf $R/gpurun_out/sprof_$TAG $R/gpurun_out/prof_$TAG
grep -i "pose_reduce\|small batch" $R/gpurun_out/sprof_top_$TAG.txt
grep -i "pose_reduce" $R/gpurun_out/kernel_stats_$TAG.csv | cut -c1-200
