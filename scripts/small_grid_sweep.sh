# Experiment (round 4; the NOF_QM_BLOCKS / NOF_UC_BLOCKS build knobs it set were temporary and are
# removed — the results fixed the grids in field_step.hip / optim.hip): grid sizes of
# k_quad_mirror and k_unscale_check at the headline, median per headline step from rocprofv3 traces.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for P in "2048 8192" "1024 2048" "4096 4096" "512 1024"; do
  set -- $P
  NOF_QM_BLOCKS=$1 NOF_UC_BLOCKS=$2 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/sg_$1 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > /tmp/sg_$1.log 2>&1 || exit 1
  python3 - $1 $2 <<'PY' | tee -a gpurun_out/small_grid_sweep.txt
import glob, sqlite3, statistics, sys
qm, uc = sys.argv[1], sys.argv[2]
c = sqlite3.connect(glob.glob(f"/tmp/sg_{qm}/**/*.db", recursive=True)[0])
rows = list(c.execute("select name,start,end from kernels order by start"))
idx = [i for i, r in enumerate(rows) if "k_prologue" in r[0]]
per = {}
for a, b in zip(idx[:-1], idx[1:]):
    seg = rows[a:b]
    if any("k_quad_mirror" in r[0] for r in seg) and b - a <= 30:
        for nm, s, e in seg:
            for k in ("k_quad_mirror", "k_unscale_check", "k_adam"):
                if k in nm:
                    per.setdefault(k, []).append(e - s)
print("qm_blocks", qm, "uc_blocks", uc, {k: round(statistics.median(v) / 1e3, 2) for k, v in per.items()})
PY
  rm -rf /tmp/sg_$1
done
