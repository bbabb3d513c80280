"""The multi-GPU driver with the HIP kernel inside: ShardedCoulKernel (openmmcoul/distributed.py) at
world size 2, one process per rank (mp.spawn, torch.distributed over gloo; both ranks on device 0 of
the one-GPU box -- the same calls RCCL runs on an 8-GPU node).  This exercises what the CPU test
(tests/test_distributed_cpu.py) replaces by a toy kernel:
  * the split-phase C-ABI calls (cf_compute_begin / _direct / _end) on device buffers,
  * the asynchronous all-reduce of the k-space buffer with the direct-space kernels launched
    while it is in flight, and the deferred energy all-reduce,
  * position re-replication after each rank moves its owned atoms (replicate_positions),
  * a kept neighbour list (skin) over several MD-like steps.
Bar: every rank's global energy and the gathered owned forces equal a one-rank evaluation of the
same positions (forces <= 2e-12 max|F| + 1e-9 kJ/mol/nm -- the one-rank cluster list rounds each
partner-side term to the 2^-34 fixed point, the per-atom full list of two ranks does not; energy
<= 1e-10 relative) and, on the first step, the oracle (exact k-sum 1e-8, grid 2.5e-6)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import Oracle  # noqa: E402
from openmmcoul import HipCalcCoulForceKernel  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402

STEPS = 3


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _system(case):
    if case == "C2":
        return ts.make("C2")
    return ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)


def _moves(n):
    rng = np.random.default_rng(21)
    return [rng.normal(scale=0.004, size=(n, 3)) for _ in range(STEPS)]


def _worker(rank, world, port, case, algo, skin, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from openmmcoul.distributed import ShardedCoulKernel
    system, force, pos, box = _system(case)
    kern = ShardedCoulKernel(system, force, 0, kspace_algo=algo, neighbor_skin=skin)
    p = torch.tensor(pos, dtype=torch.float64, device="cuda")
    moves = _moves(len(pos))
    res = []
    for s in range(STEPS):
        f = torch.zeros_like(p)
        kern.execute(p, box, f, include_energy=True)
        e = kern.energy_value()
        full = kern.replicate_positions(f.clone())   # every rank's owned forces, gathered
        res.append((e, full.cpu().numpy()))
        # each rank moves only its owned atoms; replication makes the copies identical again
        p[kern.lo:kern.hi] += torch.tensor(moves[s][kern.lo:kern.hi], device="cuda")
        kern.replicate_positions(p)
    out[rank] = (res, kern.lo, kern.hi, kern.kernel.device_errors())
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("case,algo,skin", [("C2", 2, 0.0), ("C2", 0, 0.0), ("w4k", 2, 0.1)])
def test_sharded_kernel_two_ranks_matches_one_rank_and_oracle(case, algo, skin):
    import torch.multiprocessing as mp
    system, force, pos, box = _system(case)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), case, algo, skin, out), nprocs=2, join=True)
    # one rank, same positions
    k = HipCalcCoulForceKernel(stream=torch.cuda.current_stream().cuda_stream, kspace_algo=algo).initialize(system, force)
    moves = _moves(len(pos))
    p = pos.copy()
    ref = []
    for s in range(STEPS):
        ref.append(k.execute_host(p, box))
        p = p + moves[s]
    o = Oracle(force, box).execute(pos, box)
    f_tol = 1e-8 if algo == 0 else 2.5e-6
    ranges = []
    for r in range(2):
        res, lo, hi, bits = out[r]
        assert bits == 0, (r, bits)
        ranges.append((lo, hi))
        for s, ((e, f), (e1, f1)) in enumerate(zip(res, ref)):
            assert abs(e - e1) <= 1e-10 * abs(e1) + 1e-8, (r, s, e, e1)
            assert np.abs(f - f1).max() <= 2e-12 * np.abs(f1).max() + 1e-9, (r, s, np.abs(f - f1).max())
        assert np.abs(res[0][1] - o["forces"]).max() <= f_tol
        assert abs(res[0][0] - o["energy"]) <= 1e-9 * abs(o["energy"]) + 1e-8
    assert ranges[0][0] == 0 and ranges[0][1] == ranges[1][0] and ranges[1][1] == len(pos)
