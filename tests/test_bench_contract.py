"""CPU checks of bench.py's host-side contract (no GPU): the timed region is whole
training rounds, and the roofline `traffic` / MFMA-busy figures resolve to the
committed PMC summaries of the same workload under profiles/."""
import json
import os

import bench


def test_rounds_cover_whole_training_rounds():
    # one whole round of n_step + 1 steps by default, and --steps K rounds up to whole rounds
    assert bench.rounds_for(None, 501) == (1, 501)
    assert bench.rounds_for(5, 501) == (1, 501)
    assert bench.rounds_for(501, 501) == (1, 501)
    assert bench.rounds_for(502, 501) == (2, 1002)


def test_pmc_traffic_resolves_committed_headline_summary():
    t, src = bench.pmc_traffic("k_scatter", "headline", 64)
    assert t is not None and t > 0, src
    js = json.load(open(os.path.join(bench.ROOT, src)))
    assert js["_workload"] == "headline:64"
    assert js["k_scatter"]["traffic_bytes"] == t
    # a workload without a committed PMC pass reports None and says so
    t2, why = bench.pmc_traffic("k_scatter", "headline", 7)
    assert t2 is None and "no PMC pass" in why


def test_pmc_mfma_resolves_committed_summary():
    e = bench.pmc_mfma()
    assert e is not None
    # the MLP backward, and the forward's MLP kernel (k_mlp_fwd, or k_colour with the sigma net
    # inside the encode kernel)
    assert 0.0 < e["k_mlp_bwd"]["mfma_util"] < 1.0
    assert any(0.0 < e.get(k, {}).get("mfma_util", 0.0) < 1.0 for k in ("k_mlp_fwd", "k_colour"))
    assert e["source"].startswith("profiles/")


def test_algorithmic_bytes_per_unit_match_survey():
    # SURVEY §8d per-unit figures the roofline is priced with
    assert bench.ENC_FWD_B == 588
    assert bench.GRID_BWD_B == 1100
    assert bench.MLP_FWD_FLOP == 17792


def _bench(*argv, env_extra=None):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(bench.ROOT, "bench.py"), *argv], capture_output=True,
                          text=True, env=env, timeout=300)


def test_gpus_n_launches_its_own_ranks():
    """`python bench.py --gpus N` with no launcher starts the N ranks itself (a torch.distributed.run
    child process) and prints rank 0's JSON line with n_gpus = N (launch plumbing, --dry-run: gloo,
    no GPU)."""
    p = _bench("--gpus", "2", "--dry-run")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    js = json.loads(lines[0])
    assert js["n_gpus"] == 2 and js["dry_run"]


def test_gpus_must_match_external_launcher():
    p = _bench("--gpus", "4", "--dry-run", env_extra={"WORLD_SIZE": "2", "RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr
    p = _bench("--gpus", "1", "--dry-run")
    assert p.returncode == 0 and json.loads(p.stdout.strip())["n_gpus"] == 1


def test_stalled_rank_ends_every_rank_nonzero_within_timeout():
    """a rank that stalls in the exchange must not hang the job. With the
    collective timeout at 3 s and rank 1 stalling before its second collective, `bench.py --gpus 2
    --dry-run` (the same init_distributed / exchange.collective path the training exchange takes)
    exits non-zero well inside the stall, and the failing rank names its rank, step and phase."""
    import time
    t0 = time.time()
    p = _bench("--gpus", "2", "--dry-run",
               env_extra={"NOF_DRY_RUN_STALL_RANK": "1", "NOF_COLLECTIVE_TIMEOUT_S": "3"})
    dt = time.time() - t0
    assert p.returncode != 0, p.stderr[-2000:]
    assert dt < 11.0 + 30.0, dt          # the stall is 12 s; torch.distributed.run start-up included
    assert "rank 0 step 1 phase all_reduce" in p.stderr, p.stderr[-3000:]
    assert "dry_run" not in p.stdout
