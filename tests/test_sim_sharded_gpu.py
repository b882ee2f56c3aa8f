"""configs[4] on the one GPU of the box: the sharded Monte-Carlo BLER sweep (my_sn/sim.py:79-133,
x_run_sn_polar/main.py:55-59) through the fused path (FusedAWGN + SC_Dec -> pl_sc_sim_count) with
sim_ber's windowed loop.

  * 2 ranks sharing cuda:0 over gloo (one process per rank, as torchrun launches them), each
    drawing stream rows [r * 65536, (r + 1) * 65536) at (512,1024), Eb/N0 0 ... 4 dB, with a
    block-error target that stops points mid-window: the summed counters are EXACTLY those of
    one rank simulating all 131072 rows (row0 0) -- same codewords, same stop decisions;
  * configs[4] at its stated size: 8 gloo ranks x 65536 rows = 524288 codewords per iteration,
    summed counters equal one process over the same rows;
  * the RCCL backend at world size 1 (device-tensor counter all_reduce in sim_ber; bench.py's
    barrier / timing max / BLER reduction under torch.distributed.run), and at world size 2 with
    one rank per GPU when the box has two (skipped on a one-GPU box);
  * the windowed loop equals the one-iteration loop (max_window=1) for the fused SC path and for
    an SCL decoder behind FusedAWGN (forward() + pl_count_errors);
  * the (512,1024) BLER matches the reference's measured table (x_run SC,
    bs = 8192) within 5 sigma of the two binomial samples (+ one reference count).
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EBNO = np.arange(0.0, 4.01, 0.5)  # configs[4]: Eb/N0 0-4 dB
BS = 65536
TARGET = 200_000  # block errors: points stop after 2 or 3 of max_mc_iter=4 iterations


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _sweep(rank, bs, process_group=None, max_window=None, target=TARGET, gpu=0, ebno=EBNO, max_mc_iter=4):
    import polar_amd
    from polar_amd import channel, sim
    k, n = 512, 1024
    fp = polar_amd.reference_frozen_pos(k, n)
    dec = polar_amd.SC_Dec(fp, n) if gpu == 0 else polar_amd.SC_Dec(fp, n, device=torch.device("cuda", gpu))
    model = channel.FusedAWGN(n, k, fp, dec, device=torch.device("cuda", gpu), seed=42, row0=rank * bs)
    _, _, cnt = sim.sim_ber(model, ebno, bs, max_mc_iter=max_mc_iter, target_block_errs=target, verbose=False,
                            device="cpu", process_group=process_group, return_counts=True, max_window=max_window)
    assert model.sim_kernel, "the sweep must run the fused pl_sc_sim_count path"
    return cnt.numpy()


def _worker(rank, world, port, out_dir, backend="gloo", target=TARGET):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "polar-code-pytorch-sionna_amd"))
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        # device="cpu" on purpose: sim_ber must reduce on the backend's device (RCCL: the GPU)
        cnt = _sweep(rank, BS, process_group=dist.group.WORLD, target=target)
    finally:
        dist.destroy_process_group()
    np.save(os.path.join(out_dir, f"r{rank}.npy"), cnt)


def test_two_ranks_one_gpu_equal_one_rank(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [np.load(tmp_path / f"r{i}.npy") for i in range(world)]
    np.testing.assert_array_equal(r[0], r[1])
    one = _sweep(0, world * BS)
    np.testing.assert_array_equal(r[0], one)
    blocks = one[:, 3] // (world * BS)
    assert set(blocks.tolist()) >= {2, 3}, blocks  # points stopped at different iterations
    assert (one[:, 1] >= TARGET).all() or (blocks == 4).any()


def test_configs4_eight_ranks_one_gpu_equal_one_rank(tmp_path):
    """configs[4] at its stated size: 8 ranks x 65536 rows = 524288 codewords per iteration,
    Eb/N0 0 ... 4 dB, each rank one process on cuda:0 with its shard of the keyed stream (gloo
    carries the [W, 4] counter all_reduce).  The global counters equal one process decoding all
    524288 rows per iteration (row0 0): same codewords, same stop decisions."""
    import torch.multiprocessing as mp
    world, target = 8, 4 * TARGET
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), "gloo", target), nprocs=world, join=True)
    r = [np.load(tmp_path / f"r{i}.npy") for i in range(world)]
    for i in range(1, world):
        np.testing.assert_array_equal(r[0], r[i])
    one = _sweep(0, world * BS, target=target)
    np.testing.assert_array_equal(r[0], one)
    blocks = one[:, 3] // (world * BS)
    assert len(set(blocks.tolist())) >= 2, blocks  # points stopped at different iterations
    assert int(one[0, 3]) >= world * BS


def test_rccl_world1_sim_ber_equals_no_group(tmp_path):
    """The RCCL branch on hardware: one rank, init_process_group("nccl", device_id=cuda:0); sim_ber
    keeps its [W, 4] counter block on the GPU for the device-tensor all_reduce (sim._counter_device)
    and returns exactly the counters of the same sweep without a process group."""
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(1, _free_port(), str(tmp_path), "nccl"), nprocs=1, join=True)
    got = np.load(tmp_path / "r0.npy")
    np.testing.assert_array_equal(got, _sweep(0, BS))


def test_rccl_world1_bench_line(tmp_path):
    """bench.py under torch.distributed.run with one rank and the RCCL backend (--dist forces the
    process group at world size 1): barrier, max-over-ranks timing and the BLER counter
    all_reduce run over RCCL; the JSON line is the single-GPU one."""
    import json
    import subprocess
    import sys
    env = dict(os.environ, PL_BENCH_BACKEND="nccl")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"), "--dist",
           "--steps", "50", "--warmup", "5", "--no-cpu-baseline", "--no-sim-iteration", "--no-configs"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["config"]["parallelism"] == "dp1" and line["dist_backend"] == "nccl"
    assert line["value"] > 10.0 and line["bler"] > 0.5


def _worker_per_gpu(rank, world, port, out_dir):
    """One rank per GPU over RCCL (xGMI): rank r on cuda:r, its shard of the keyed stream (rows
    [r * BS, (r + 1) * BS)), one SNR point; sim_ber's [W, 4] counter all_reduce runs on the device."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "polar-code-pytorch-sionna_amd"))
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    try:
        cnt = _sweep(rank, BS, process_group=dist.group.WORLD, gpu=rank, ebno=np.array([3.0]), max_mc_iter=2)
    finally:
        dist.destroy_process_group()
    np.save(os.path.join(out_dir, f"r{rank}.npy"), cnt)


two_gpus = pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (RCCL over xGMI)")


@two_gpus
def test_rccl_two_gpus_sim_ber_equals_one_rank(tmp_path):
    """RCCL at world size 2, one process per GPU (my_sn/sim.py:72-97, stop rule
    :107-133 -- the counters the harness reduces).  Both ranks end with the same global counters,
    equal to one process simulating both shards' rows on one GPU."""
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_worker_per_gpu, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [np.load(tmp_path / f"r{i}.npy") for i in range(world)]
    np.testing.assert_array_equal(r[0], r[1])
    one = _sweep(0, world * BS, ebno=np.array([3.0]), max_mc_iter=2)
    np.testing.assert_array_equal(r[0], one)


@two_gpus
def test_rccl_two_gpus_bench_line(tmp_path):
    """bench.py as the driver launches it at --gpus 2 (torch.distributed.run, one rank per GPU,
    the default RCCL backend): the line reports both GPUs and the RCCL backend, and the value is
    the whole job's throughput."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k != "PL_BENCH_BACKEND"}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "50", "--warmup", "5", "--no-cpu-baseline", "--no-sim-iteration", "--no-configs"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["dist_backend"] == "nccl" and line["config"]["parallelism"] == "dp2"
    assert line["config"]["global_batch"] == 2 * line["config"]["bs_per_gpu"]
    assert line["value"] > 10.0 and line["bler"] > 0.5


def test_window_equals_sequential_fused():
    a = _sweep(0, 16384)
    b = _sweep(0, 16384, max_window=1)
    np.testing.assert_array_equal(a, b)


def test_window_equals_sequential_scl_forward():
    import polar_amd
    from polar_amd import channel, sim
    k, n = 128, 256
    fp = polar_amd.reference_frozen_pos(k, n)
    res = []
    for w in (None, 1):
        model = channel.FusedAWGN(n, k, fp, polar_amd.SCL_Dec(fp, n, 4, device="cuda"), seed=5)
        assert model.error_counts(16, 1.0) is None  # SCL: forward() + pl_count_errors
        _, _, c = sim.sim_ber(model, np.array([1.0, 2.0, 3.0]), 512, max_mc_iter=7, target_block_errs=300,
                              verbose=False, device="cuda", return_counts=True, max_window=w)
        res.append(c.numpy())
    np.testing.assert_array_equal(res[0], res[1])


REF_BLER_1024 = {2.0: .9999, 2.5: .9954, 3.0: .9735, 3.5: .8981, 4.0: .7612, 4.5: .5254}


def test_bler_matches_reference_table_512_1024():
    import polar_amd
    from polar_amd import channel, sim
    k, n = 512, 1024
    fp = polar_amd.reference_frozen_pos(k, n)
    model = channel.FusedAWGN(n, k, fp, polar_amd.SC_Dec(fp, n), seed=1234)
    pts = np.array(sorted(REF_BLER_1024))
    _, bler, c = sim.sim_ber(model, pts, BS, max_mc_iter=2, verbose=False, device="cuda", return_counts=True)
    n_ref = 8192
    for i, e in enumerate(pts):
        p_ref, p = REF_BLER_1024[e], float(bler[i])
        n_ours = int(c[i, 3])
        assert n_ours == 2 * BS
        q = (p_ref * n_ref + p * n_ours) / (n_ref + n_ours)
        sigma = np.sqrt(q * (1 - q) * (1 / n_ref + 1 / n_ours))
        assert abs(p - p_ref) <= 5 * sigma + 1 / n_ref, (e, p, p_ref, sigma)
