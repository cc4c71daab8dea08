"""Multi-rank path: env sharding by global id, no data-path collective.

world_size-2 gloo runs of tests/dist_worker.py (each rank a separate process, as under
torch.distributed.run) must reproduce, bit for bit, one process stepping the whole batch.  The CPU
variant shards the oracle; the gpu variant shards the HIP product path (both ranks on cuda:0 — the
point is the id-keyed sharding, not the card count).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from marllb_amd import dist as lbdist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from dist_worker import actions  # noqa: E402

B, S, T, SEED = 24, 4, 4, 1234


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(mode: str, world: int, out: str):
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(HERE, "dist_worker.py"), "--mode", mode,
             "--port", str(port), "--out", out, "--batch", str(B), "--servers", str(S),
             "--steps", str(T), "--seed", str(SEED)], env=env))
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=240))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert rcs == [0] * world, rcs
    return np.load(out)


def single_process_reference(oracle_mod, world: int):
    from marllb_amd.env import make_config
    n = world * B
    env = oracle_mod.OracleEnv(make_config(n, S, seed=SEED, max_steps=1000), threads=2)
    gids = np.arange(n, dtype=np.int64)
    obs, rew = [env.reset()], []
    for k in range(T):
        o, r, _, _ = env.step(actions(gids, S, k))
        obs.append(o)
        rew.append(r)
    return np.stack(obs), np.stack(rew)


def test_shard_arithmetic():
    sh = lbdist.Shard(rank=3, world=8, envs_per_rank=65536)
    assert sh.env_id_offset == 3 * 65536 and sh.global_envs == 8 * 65536
    assert list(sh.global_ids())[:2] == [196608, 196609]
    assert lbdist.throughput(sh, 10, 2.0) == 8 * 65536 * 10 / 2.0
    assert lbdist.max_over_ranks(1.5) == 1.5  # no process group: identity
    assert lbdist.gather_over_ranks(1.5) == [1.5]


@pytest.mark.parametrize("world", [2, 4])
def test_rank_oracle_shards_equal_single_process(tmp_path, oracle_mod, world):
    res = run_ranks("oracle", world, str(tmp_path / "r.npz"))
    assert list(res["offsets"]) == [r * B for r in range(world)]
    assert float(res["slowest"]) == float(world)
    assert float(res["rate"]) == world * B * T / float(world)
    assert list(res["per_rank"]) == [float(r + 1) for r in range(world)]  # rank order
    obs, rew = single_process_reference(oracle_mod, world)
    np.testing.assert_array_equal(res["obs"], obs)
    np.testing.assert_array_equal(res["rew"], rew)


@pytest.mark.gpu
def test_two_rank_gpu_shards_equal_single_process_oracle(tmp_path, oracle_mod):
    res = run_ranks("gpu", 2, str(tmp_path / "g.npz"))
    obs, rew = single_process_reference(oracle_mod, 2)
    np.testing.assert_array_equal(res["obs"], obs)
    np.testing.assert_array_equal(res["rew"], rew)


@pytest.mark.gpu
@pytest.mark.parametrize("world,batch", [(2, 2048), (8, 512)])
def test_bench_self_launches_ranks(world, batch):
    """`bench.py --gpus N` without torchrun starts its own N rank processes (the driver's
    multi-GPU contract, rehearsed up to the 8 ranks of one node); gloo for the measurement
    collectives so every rank may share one card.  Rank 0 prints exactly one JSON line with
    n_gpus = N and the global batch of all shards."""
    import json
    root = os.path.dirname(HERE)
    env = dict(os.environ, LBSIM_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world),
                        "--steps", "3", "--warmup", "1", "--batch", str(batch),
                        "--no-cpu-baseline", "--no-graph", "--prewarm-ms", "0"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["config"]["global_batch"] == world * batch
    assert out["value"] > 0
    ranks = out["ranks"]
    assert ranks["world_size"] == world and len(ranks["elapsed_s"]) == world
    assert ranks["elapsed_min_s"] <= ranks["elapsed_max_s"]
    assert abs(ranks["elapsed_max_s"] - out["ms_per_step"] * 3 / 1e3) < 1e-9


@pytest.mark.gpu
def test_bench_torchrun_rccl_world1():
    """The driver's multi-GPU launch form (`python -m torch.distributed.run --nproc-per-node N
    ... bench.py --gpus N`) at N = 1 on the one card a test box has: torchrun's environment
    contract gives the rank, bench.py opens an RCCL ("nccl") process group with device_id, and the
    timing barrier plus max_over_ranks / gather_over_ranks run as RCCL collectives on a device
    tensor -- the code path of the 8-GPU scaling run, executed end to end."""
    import json
    root = os.path.dirname(HERE)
    env = {k: v for k, v in os.environ.items() if k != "LBSIM_DIST_BACKEND"}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "1", "--master-addr", "127.0.0.1", "--master-port",
                        str(free_port()), os.path.join(root, "bench.py"), "--gpus", "1",
                        "--steps", "3", "--warmup", "1", "--batch", "2048", "--no-cpu-baseline",
                        "--no-graph", "--prewarm-ms", "0"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["value"] > 0
    ranks = out["ranks"]
    assert ranks["backend"] == "nccl" and ranks["world_size"] == 1
    assert len(ranks["elapsed_s"]) == 1
    assert abs(ranks["elapsed_max_s"] - out["ms_per_step"] * 3 / 1e3) < 1e-9


@pytest.mark.gpu
def test_bench_graph_leg_runs_in_a_child_process():
    """The graph leg runs in a child process (bench.graph_leg_child): the headline line carries
    its result, marked as a child's, and the headline process never captures a graph."""
    import json
    root = os.path.dirname(HERE)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "5",
                        "--warmup", "2", "--batch", "2048", "--no-cpu-baseline", "--prewarm-ms", "0"],
                       cwd=root, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    g = json.loads(lines[0])["graph"]
    assert "error" not in g, g
    assert g["process"].startswith("child") and g["value"] > 0 and g["autoreset"] == "next_step"
