# Experiment (round 4; the NOF_ADAM_BLOCKS override it set was a temporary build knob, now removed:
# the cap is fixed at 4096 in optim.hip): k_adam grid size at the headline, kernel time from rocprofv3 traces
# (summarised on the box: median k_adam duration over the headline steps).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for B in 8192 4096 2048 1024; do
  NOF_ADAM_BLOCKS=$B timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/adam_$B -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > /tmp/adam_$B.log 2>&1 || exit 1
  python3 - $B <<'PY' | tee -a gpurun_out/adam_blocks_sweep.txt
import glob, sqlite3, statistics, sys
B = sys.argv[1]
c = sqlite3.connect(glob.glob(f"/tmp/adam_{B}/**/*.db", recursive=True)[0])
rows = list(c.execute("select name,start,end from kernels order by start"))
idx = [i for i, r in enumerate(rows) if "k_prologue" in r[0]]
per = []
for a, b in zip(idx[:-1], idx[1:]):
    seg = rows[a:b]
    if any("k_quad_mirror" in r[0] for r in seg) and b - a <= 30:
        per += [e - s for nm, s, e in seg if "k_adam" in nm]
print("adam_blocks", B, "median_us", round(statistics.median(per) / 1e3, 2), "n", len(per))
PY
  rm -rf /tmp/adam_$B
done
