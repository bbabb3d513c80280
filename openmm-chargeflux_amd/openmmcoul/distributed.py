"""Atom decomposition over GPUs (one process per GPU, torch.distributed over RCCL).

The reference is single-device (platforms/cuda/src/CudaCoulKernelFactory.cpp:40 binds
contexts[0]); this is new.  The only data-path exchange is the structure factor S(k):
every rank sums S over its owned atoms, one all-reduce (sum) makes it global, and the
rest of the evaluation (reciprocal forces, direct space with a full neighbour list,
exclusions, chain rule) is local to the owned, molecule-aligned atom range
(SURVEY.md §8(e)).  Positions are replicated; an MD driver re-replicates them after
integrating its owned atoms (`replicate_positions`).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .kernel import HipCalcCoulForceKernel


class _DeviceArray:
    """Zero-copy view of a raw device pointer for torch (CUDA array interface)."""

    def __init__(self, ptr: int, count: int):
        self.__cuda_array_interface__ = {"shape": (count,), "typestr": "<f8", "data": (ptr, False), "version": 2,
                                         "strides": None}


def device_buffer_as_tensor(ptr: int, count: int, device) -> torch.Tensor:
    return torch.as_tensor(_DeviceArray(ptr, count), device=device)


class ShardedCoulKernel:
    """CalcCoulForceKernel over `world_size` ranks.  execute() returns the GLOBAL energy
    (device scalar) and adds forces for this rank's owned atoms into `forces`."""

    def __init__(self, system, force, device: int, group=None, kspace_algo: int = 0, kernel=None,
                 neighbor_skin: float = 0.0, grid_width: int = 0, precision: str = "double", **options):
        """options: further HipCalcCoulForceKernel options (pair_list, handover, variants, ...)."""
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if kernel is None:
            self.device = torch.device("cuda", device)
            stream = torch.cuda.current_stream(self.device).cuda_stream
            kernel = HipCalcCoulForceKernel(device=device, stream=stream, rank=self.rank, world_size=self.world,
                                            kspace_algo=kspace_algo, grid_width=grid_width,
                                            precision=precision, **options).initialize(system, force)
            if neighbor_skin > 0:
                kernel.set_neighbor_skin(neighbor_skin)
        else:  # any object with the split-phase kernel interface (tests drive this on CPU/gloo)
            self.device = torch.device(device) if not isinstance(device, torch.device) else device
        self.kernel = kernel
        self.lo, self.hi = self.kernel.owned_range()
        # two energy buffers: the scalar all-reduce of one evaluation is left in flight (the
        # compute stream does not wait for it) and completed before its buffer is reused, or
        # when the caller asks for the value (energy_value / synchronize)
        self._ebufs = [torch.zeros(1, dtype=torch.float64, device=self.device) for _ in range(2)]
        self._ework = [None, None]
        self._ecur = 0
        self.energy = self._ebufs[0]
        self._sbuf = self.kernel.kspace_tensor(self.device)
        self._gidx = None
        if self.world > 1:
            # every rank's owned range -> padded all-gather layout for position replication
            mine = torch.tensor([self.lo, self.hi], dtype=torch.int64, device=self.device)
            allr = [torch.zeros_like(mine) for _ in range(self.world)]
            dist.all_gather(allr, mine, group=self.group)
            ranges = [tuple(int(v) for v in t.cpu()) for t in allr]
            self._maxown = max(1, max(h - l for l, h in ranges))
            rows = []
            for r, (l, h) in enumerate(ranges):
                rows.extend(range(r * self._maxown, r * self._maxown + (h - l)))
            self._gidx = torch.tensor(rows, dtype=torch.int64, device=self.device)
            self._send = torch.zeros(self._maxown, 3, dtype=torch.float64, device=self.device)
            self._recv = torch.zeros(self.world * self._maxown, 3, dtype=torch.float64, device=self.device)

    def execute(self, positions: torch.Tensor, box, forces: torch.Tensor | None, include_energy: bool = True):
        k = self.kernel
        if self.world == 1 and hasattr(k, "execute_device"):
            # one rank: a single cf_compute call (graph-replayable, cf_set_graph) into one energy buffer
            self.energy = self._ebufs[0]
            k.execute_device(positions, box, forces is not None, include_energy, forces, self.energy)
            return self.energy
        k.begin(positions, box, forces is not None, include_energy)
        if self.world > 1 and self._sbuf is not None:
            # the direct-space kernels do not need S(k): they run while it is all-reduced
            work = dist.all_reduce(self._sbuf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            if hasattr(k, "direct"):
                k.direct()
            work.wait()
        i = self._ecur = 1 - self._ecur
        if self._ework[i] is not None:
            self._ework[i].wait()
            self._ework[i] = None
        self.energy = self._ebufs[i]
        k.end(forces, self.energy)
        if self.world > 1 and include_energy:
            self._ework[i] = dist.all_reduce(self.energy, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        return self.energy

    def synchronize(self):
        """Complete the energy reductions still in flight (before reading an energy)."""
        for i, w in enumerate(self._ework):
            if w is not None:
                w.wait()
                self._ework[i] = None

    def energy_value(self) -> float:
        self.synchronize()
        return self.energy.item()

    def replicate_positions(self, positions: torch.Tensor):
        """After each rank updated positions[lo:hi], make every rank's copy identical
        (one all-gather of the owned slices, padded to the largest)."""
        if self.world == 1:
            return positions
        p = positions.view(-1, 3)
        self._send[: self.hi - self.lo].copy_(p[self.lo:self.hi])
        if dist.get_backend(self.group) == "gloo":   # gloo has no all_gather_into_tensor
            dist.all_gather(list(self._recv.view(self.world, self._maxown, 3).unbind(0)), self._send, group=self.group)
        else:
            dist.all_gather_into_tensor(self._recv, self._send, group=self.group)
        torch.index_select(self._recv, 0, self._gidx, out=p)
        return positions
