"""Multi-rank harness path on CPU (gloo, world_size 2): the RCCL code path with the gloo backend.

Each rank simulates its own shard (seed 42 + rank); the only exchange is the all_reduce(SUM) of
the int64[4] counters per Monte-Carlo iteration (my_sn/sim.py:72-97 semantics).  Checks: every
rank returns identical global BER/BLER, and the global counters equal the sum of what each rank
counts when it runs alone with the same seed.  Decoding uses the oracle (checker) - no GPU here.
"""
import os
import socket

import numpy as np
import pytest
import torch as tc
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model(rank):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "polar-code-pytorch-sionna_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from polar_amd import channel, frozen
    from test_harness import _OracleDecoder
    G, _, fp = frozen.get_Kern_frozen_bits(64, 32, frozen.F2)
    fp = frozen.reference_frozen_pos(32, 64)
    return channel.System_AWGN_model(64, 32, channel.DenseEncoder(fp, 64, G), _OracleDecoder(fp.numpy()))


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from polar_amd import sim
    ebno = np.array([0.0, 1.0, 2.0])
    tc.manual_seed(42 + rank)
    ber, bler, cnt = sim.sim_ber(_model(rank), ebno, 40, max_mc_iter=3, verbose=False,
                                 process_group=dist.group.WORLD, return_counts=True)
    dist.destroy_process_group()
    tc.manual_seed(42 + rank)
    _, _, local = sim.sim_ber(_model(rank), ebno, 40, max_mc_iter=3, verbose=False, return_counts=True)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), ber=ber.numpy(), bler=bler.numpy(), cnt=cnt.numpy(),
             local=local.numpy())


def test_two_rank_counters_allreduce(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [np.load(tmp_path / f"r{i}.npz") for i in range(world)]
    np.testing.assert_array_equal(r[0]["ber"], r[1]["ber"])
    np.testing.assert_array_equal(r[0]["bler"], r[1]["bler"])
    np.testing.assert_array_equal(r[0]["cnt"], r[0]["local"] + r[1]["local"])
    assert (r[0]["cnt"][:, 3] == 2 * 40 * 3).all()  # every rank ran every iteration
    assert (r[0]["cnt"][:, 1] > 0).all()


def _keyed_worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "polar-code-pytorch-sionna_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from polar_amd import sim
    from test_sim_window import KeyedModel
    bs = 12
    m = KeyedModel(row0=rank * bs, rows_total=world * bs)
    _, _, cnt = sim.sim_ber(m, np.array([0.0, 2.0, 4.0, 7.0]), bs, max_mc_iter=9, target_block_errs=30,
                            verbose=False, process_group=dist.group.WORLD, return_counts=True)
    dist.destroy_process_group()
    np.savez(os.path.join(out_dir, f"k{rank}.npz"), cnt=cnt.numpy())


def test_two_rank_windowed_shards_equal_one_rank(tmp_path):
    """Windowed sim_ber over 2 gloo ranks, each drawing its rows of the keyed stream: the global
    counters equal one rank simulating all rows (same codewords, same stop decisions)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from polar_amd import sim
    from test_sim_window import KeyedModel
    world = 2
    mp.spawn(_keyed_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [np.load(tmp_path / f"k{i}.npz")["cnt"] for i in range(world)]
    np.testing.assert_array_equal(r[0], r[1])
    _, _, one = sim.sim_ber(KeyedModel(), np.array([0.0, 2.0, 4.0, 7.0]), world * 12, max_mc_iter=9,
                            target_block_errs=30, verbose=False, return_counts=True)
    np.testing.assert_array_equal(r[0], one.numpy())
    assert (r[0][:, 3] % (world * 12) == 0).all() and r[0][0, 1] >= 30


def test_cli_parses_reference_flags():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "polar-code-pytorch-sionna_amd"))
    from polar_amd import cli
    c = cli.parse(["--k", "32", "--n", "64", "--algos", "[scl]", "--bs", "100", "--mc_iter", "1"])
    assert (c.k, c.n, c.algos, c.bs, c.mc_iter, c.list_size, c.snr_end) == (32, 64, ["scl"], 100, 1, 8, 5)
