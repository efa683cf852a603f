# Round-4 profiles: headline (scripts/gpu_prof_r3.sh: kernel-trace summary + PMC traffic / MFMA / SQ
# passes) and the NerfRunner.train()-sized step (scripts/gpu_small_prof.sh). Usage: bash scripts/gpu_prof_r4.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r4}
bash $R/scripts/gpu_prof_r3.sh $TAG || exit $?
bash $R/scripts/gpu_small_prof.sh $TAG > $R/gpurun_out/sprof_top_$TAG.txt 2>&1 || { tail -20 $R/gpurun_out/sprof_top_$TAG.txt; exit 9; }
cp $R/gpurun_out/sprof_$TAG/run_kernel_stats.csv $R/gpurun_out/kernel_stats_parity_$TAG.csv
rm -rf $R/gpurun_out/sprof_$TAG $R/gpurun_out/prof_$TAG
echo profiles done
