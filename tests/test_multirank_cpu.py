"""World-size-2 gloo run of the multi-GPU host logic on CPU: range shards of the
global sweep are disjoint and complete, and the barrier / max-over-ranks timing
used by bench.py works over torch.distributed (gloo, 127.0.0.1)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as tmp  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, ws, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws), LOCAL_RANK=str(rank))
    import bench
    from noisyquantumsimulator_amd import engine as E
    from noisyquantumsimulator_amd import sweeps as SW
    w, r, local, pg = bench._dist()
    assert (w, r, local) == (ws, rank, rank)
    b = SW.c2_rank_shard(rank, ws)
    p = E.pack_params(b)
    keys = np.stack([p[0], p[1]])            # (Omega, Delta) identify a point
    gathered = [None] * ws
    dist.all_gather_object(gathered, keys)
    bench._barrier(pg)
    t = bench._max_over_ranks(pg, float(rank + 1))
    if rank == 0:
        out.put((gathered, t))
    dist.destroy_process_group()


def test_two_rank_sharding_and_timing():
    ws = 2
    port = _free_port()
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for pr in procs:
        pr.start()
    gathered, tmax = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert tmax == 2.0
    from noisyquantumsimulator_amd import engine as E
    from noisyquantumsimulator_amd import sweeps as SW
    full = SW.omega_delta_grid(100, 200)
    pf = E.pack_params(full)
    allk = np.concatenate(gathered, axis=1)
    assert allk.shape[1] == 20_000 == full.n
    a = set(map(tuple, allk.T.round(6)))
    b = set(map(tuple, np.stack([pf[0], pf[1]]).T.round(6)))
    assert a == b and len(a) == 20_000      # disjoint and complete


@pytest.mark.parametrize("ws", [1, 2, 3, 8])
def test_c4_range_shards_are_exact_partition(ws):
    """C4 strong-scaling partition: concatenating the ranks' derived shards reproduces
    the full grid's derivation bit for bit (every derived quantity is per point)."""
    from noisyquantumsimulator_amd import engine as E
    from noisyquantumsimulator_amd import sweeps as SW
    n_T, n_P = 7, 5
    n = 2 * n_T * n_P
    full = E.pack_params(SW.species_temperature_power_grid(n_T, n_P))
    parts = [E.pack_params(SW.species_temperature_power_grid(
        n_T, n_P, point_slice=SW.range_shard(n, r, ws))) for r in range(ws)]
    assert sum(p.shape[1] for p in parts) == n
    np.testing.assert_array_equal(np.concatenate(parts, axis=1), full)


def test_c4_grid_layout():
    from noisyquantumsimulator_amd import sweeps as SW
    assert SW.C4_POINTS == 1_000_000
    idx = np.array([0, 499_999, 500_000, 999_999])
    b = SW.species_temperature_power_grid(point_index=idx)
    assert b.n == 4
    # species-major: Rb87 (first half) then Cs133 (second half) -> different masses
    assert b["mass"][0] == b["mass"][1] != b["mass"][2] == b["mass"][3]
