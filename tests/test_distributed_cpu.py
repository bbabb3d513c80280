"""World-size-2 gloo tests (CPU) of the multi-GPU driver: the molecule-aligned atom
decomposition (cf_partition, host-only C-ABI) and ShardedCoulKernel's split-phase
orchestration (begin -> all-reduce S(k) -> end -> all-reduce energy; position
re-replication).  The HIP kernel needs a GPU, so the split-phase kernel is replaced by a
CPU toy with the same contract: partial structure factors over owned atoms in `begin`,
global S after the all-reduce, owned-atom forces and a per-rank energy in `end`."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from openmmcoul import _cabi
from openmmcoul import testsystems as ts


def _partition(force, box, world):
    lib = _cabi.load_library()
    import ctypes as C
    p, keep = force.to_cparams(box)
    out = []
    for r in range(world):
        lo, hi = C.c_int32(), C.c_int32()
        _cabi.check(lib.cf_partition(C.byref(p), world, r, C.byref(lo), C.byref(hi)), lib)
        out.append((lo.value, hi.value))
    return out


def test_partition_covers_and_never_splits_molecules():
    system, force, pos, box = ts.water_box(301, cutoff=0.6, every_bond_angle=4)
    n = force.getNumParticles()
    for world in (1, 2, 3, 4, 7, 8):
        ranges = _partition(force, box, world)
        assert ranges[0][0] == 0 and ranges[-1][1] == n
        for (a, b), (c, d) in zip(ranges, ranges[1:]):
            assert b == c and a <= b
        for lo, hi in ranges:
            assert lo % 3 == 0 and hi % 3 == 0  # water boundaries
        sizes = [hi - lo for lo, hi in ranges]
        assert max(sizes) - min(sizes) <= 6


def test_partition_rejects_bad_input():
    f = ts.water_box(10, cutoff=0.3)[1]
    f.addException(0, 10 ** 6)
    with pytest.raises(_cabi.ChargeFluxError) as ei:
        _partition(f, np.eye(3), 2)
    assert ei.value.code == _cabi.CF_ERR_INVALID


class ToyKernel:
    """CPU stand-in with the split-phase contract of HipCalcCoulForceKernel."""

    def __init__(self, pos, q, box, lo, hi, rank):
        L = np.diag(box)
        ks = [(a, b, c) for a in range(0, 3) for b in range(-2, 3) for c in range(-2, 3) if (a, b, c) > (0, 0, 0)]
        self.k = torch.tensor([[2 * np.pi * a / L[0], 2 * np.pi * b / L[1], 2 * np.pi * c / L[2]] for a, b, c in ks],
                              dtype=torch.float64)
        self.w = torch.exp(-(self.k ** 2).sum(1) / 4.0) / (self.k ** 2).sum(1)
        self.q = torch.tensor(q)
        self.lo, self.hi, self.rank = lo, hi, rank
        self.S = torch.zeros(2 * len(ks), dtype=torch.float64)

    def owned_range(self):
        return self.lo, self.hi

    def kspace_tensor(self, device):
        return self.S

    def begin(self, pos, box, forces, energy):
        g = pos[self.lo:self.hi] @ self.k.T
        q = self.q[self.lo:self.hi, None]
        K = len(self.w)
        self.S[:K] = (q * torch.cos(g)).sum(0)
        self.S[K:] = (q * torch.sin(g)).sum(0)
        self._pos = pos

    def end(self, forces, energy):
        K = len(self.w)
        cs, ss = self.S[:K], self.S[K:]
        g = self._pos[self.lo:self.hi] @ self.k.T
        q = self.q[self.lo:self.hi, None]
        coef = 2 * self.w * (cs * torch.sin(g) - ss * torch.cos(g)) * q
        if forces is not None:
            forces[self.lo:self.hi] += coef @ self.k
        e = (self.w * (cs ** 2 + ss ** 2)).sum() if self.rank == 0 else torch.zeros((), dtype=torch.float64)
        energy.fill_(float(e) + float((q ** 2).sum()) * -0.1)


def _worker(rank, world, port, pos, q, box, ranges, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from openmmcoul.distributed import ShardedCoulKernel
    lo, hi = ranges[rank]
    kern = ShardedCoulKernel(None, None, "cpu", kernel=ToyKernel(pos, q, box, lo, hi, rank))
    p = torch.tensor(pos)
    f = torch.zeros_like(p)
    e = kern.execute(p, box, f, include_energy=True)
    e = kern.energy_value()   # the energy all-reduce is left in flight by execute
    # a second evaluation uses the other energy buffer; the first value must be untouched
    f2 = torch.zeros_like(p)
    kern.execute(p, box, f2, include_energy=True)
    assert kern.energy_value() == e and torch.equal(f2, f)
    # owned forces -> gather all ranks' owned slices through the position re-replication path
    full = kern.replicate_positions(f.clone())
    # a rank moves only its owned atoms; replication must make every copy identical
    p2 = p.clone()
    p2[lo:hi] += 0.01 * (rank + 1)
    kern.replicate_positions(p2)
    out[rank] = (float(e), full.numpy().copy(), p2.numpy().copy())
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_sharded_driver_two_ranks_gloo():
    system, force, pos, box = ts.water_box(40, cutoff=0.5, every_bond_angle=3)
    q = force.arrays()["charges"]
    n = len(pos)
    # single-rank reference
    ref = ToyKernel(pos, q, box, 0, n, 0)
    p = torch.tensor(pos)
    ref.begin(p, box, True, True)
    f_ref = torch.zeros_like(p)
    e_ref = torch.zeros(1, dtype=torch.float64)
    ref.end(f_ref, e_ref)
    ranges = _partition(force, box, 2)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), pos, q, box, ranges, out), nprocs=2, join=True)
    for r in range(2):
        e, f, p2 = out[r]
        assert e == pytest.approx(float(e_ref), rel=1e-12)
        assert np.abs(f - f_ref.numpy()).max() < 1e-10
        expect = pos.copy()
        for rr, (lo, hi) in enumerate(ranges):
            expect[lo:hi] += 0.01 * (rr + 1)
        assert np.abs(p2 - expect).max() < 1e-14
