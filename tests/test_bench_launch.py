"""bench.py --gpus N as its own launcher: without WORLD_SIZE in the environment
it starts N fresh rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, as
torch.distributed.run would), waits for all of them and relays rank 0's JSON line; a failing rank
fails the run.  --dry-run does the rendezvous and the max / sum reductions over gloo with no GPU."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


@pytest.mark.parametrize("n", [2, 3, 8])   # 8: the driver's 8-GPU node, rehearsed over gloo
def test_bench_spawns_n_ranks_dry_run(n):
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--steps", "7", "--warmup", "1", "--dry-run"],
                       cwd=REPO, env=_env(CUDA_VISIBLE_DEVICES=""), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout           # exactly one JSON line, from rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["config"]["chains"] == n and d["steps"] == 7
    # sum over ranks of 10·(r+1) leapfrogs, max over ranks of 1 ms·(r+1)
    assert d["leapfrogs"] == 10.0 * n * (n + 1) / 2
    assert abs(d["t_max"] - 0.001 * n) < 1e-12
    # both aggregates of the N-GPU line from the gathered per-rank numbers (bench.aggregate_ranks):
    # makespan Σ lf / max t and chain throughput Σ lf_r / t_r, each × P = 7850
    rk = d["ranks"]
    assert rk["per_rank_leapfrogs"] == [10.0 * (r + 1) for r in range(n)]
    assert rk["per_rank_ms"] == pytest.approx([1.0 * (r + 1) for r in range(n)])
    assert rk["value_makespan"] == pytest.approx(10.0 * n * (n + 1) / 2 / (0.001 * n) * 7850)
    assert rk["value_chain_throughput"] == pytest.approx(n * 10000.0 * 7850)
    envs = d["rank_env"]
    assert [e["RANK"] for e in envs] == [str(r) for r in range(n)]
    assert [e["LOCAL_RANK"] for e in envs] == [str(r) for r in range(n)]
    assert all(e["WORLD_SIZE"] == str(n) and e["MASTER_ADDR"] == "127.0.0.1" for e in envs)
    assert len({e["MASTER_PORT"] for e in envs}) == 1


def test_bench_launcher_fails_when_a_rank_fails():
    # --path is validated by argparse in every child: all ranks exit 2 → the launcher exits non-zero
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--path", "bogus", "--dry-run"],
                       cwd=REPO, env=_env(CUDA_VISIBLE_DEVICES=""), capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_respects_external_launcher_env():
    # WORLD_SIZE already set (torchrun / the driver): bench.py is one rank and does not spawn
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, "bench.py", "--gpus", "2", "--dry-run"], cwd=REPO,
                              env=_env(CUDA_VISIBLE_DEVICES="", RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2",
                                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=240) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-2000:] for o in outs]
    d = json.loads([ln for ln in outs[0][0].splitlines() if ln.startswith("{")][-1])
    assert d["n_gpus"] == 2 and not [ln for ln in outs[1][0].splitlines() if ln.startswith("{")]


def test_aggregate_ranks_hand_computed():
    sys.path.insert(0, REPO)
    import bench
    per = [{"leapfrogs": 182, "seconds": 1.70e-3}, {"leapfrogs": 234, "seconds": 2.11e-3}]
    a = bench.aggregate_ranks(per, P_dim=1)
    assert a["value_makespan"] == pytest.approx((182 + 234) / 2.11e-3)
    assert a["value_chain_throughput"] == pytest.approx(182 / 1.70e-3 + 234 / 2.11e-3)
    assert a["per_rank_leapfrogs"] == [182.0, 234.0]


def test_predicted_scaling_uses_the_device_schedule():
    """The host twin of the Philox schedule gives chains 0-7 the timed leapfrogs of the driver's shape
    (--steps 20 --warmup 5); chain 0's 182 is what BENCH_r04 measured on the GPU."""
    sys.path.insert(0, REPO)
    import bench
    pr = bench.predicted_scaling(5, 20)
    assert pr["chain_leapfrogs"] == [182, 159, 196, 183, 148, 198, 234, 198]
    assert pr["1"]["makespan"] == pytest.approx(1.0) and pr["1"]["chain_throughput"] == pytest.approx(1.0)
    # makespan is held back by the slowest chain (234 leapfrogs); chain throughput is not
    assert 6.0 < pr["8"]["makespan"] < 7.2 and 7.5 < pr["8"]["chain_throughput"] < 8.5
