"""The single-rank reciprocal chain on a second stream: bin sort, spread,
DFTs, coefficients and interpolation run beside the cell list and direct space, joined before
k_assemble_energy, which folds the reciprocal dE/dq and forces in the one-stream order.  Bar:
bitwise equality with cf_set_overlap(h, 0) (one stream) for energy, forces, dE/dq and the energy
terms, with and without a kept list, energy-only calls in between, and graph replay -- for both
hand-over forms (cf_options.handover: events, the default, and the opt-in stream-memory waits)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from openmmcoul import HipCalcCoulForceKernel  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _run(overlap, system, force, pos, box, skin, graph=False, steps=4, handover="event", variants=0):
    stream = torch.cuda.current_stream().cuda_stream
    k = HipCalcCoulForceKernel(stream=stream, kspace_algo=2, handover=handover,
                               variants=variants).initialize(system, force)
    k.set_overlap(overlap)
    if skin:
        k.set_neighbor_skin(skin)
    if graph:
        k.set_graph(True)
    rng = np.random.default_rng(9)
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    out = []
    for s in range(steps):
        f = torch.zeros_like(pt)
        e = torch.zeros(1, dtype=torch.float64, device="cuda")
        forces = s != 2   # an energy-only evaluation in between
        k.execute_device(pt, box, forces, True, f, e)
        torch.cuda.synchronize()
        out.append((e.item(), f.cpu().numpy(), k.dedq() if forces else None, k.energy_terms()))
        pt += torch.tensor(rng.normal(scale=0.004, size=pos.shape), device="cuda")
    k.destroy()
    return out


@pytest.mark.parametrize("handover", ["event", "memory"])
@pytest.mark.parametrize("skin,graph", [(0.0, False), (0.1, False), (0.1, True)])
def test_overlap_is_bitwise_one_stream(skin, graph, handover):
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    a = _run(True, system, force, pos, box, skin, graph, handover=handover)
    b = _run(False, system, force, pos, box, skin, graph)
    for (ea, fa, da, ta), (eb, fb, db, tb) in zip(a, b):
        assert ea == eb and np.array_equal(fa, fb) and np.array_equal(ta, tb)
        assert (da is None and db is None) or np.array_equal(da, db)


def test_overlap_c2_matches_oracle():
    from oracle import Oracle
    system, force, pos, box = ts.make("C2")
    k = HipCalcCoulForceKernel(kspace_algo=2).initialize(system, force)
    e, f = k.execute_host(pos, box)
    ref = Oracle(force, box).execute(pos, box)
    assert np.abs(f - ref["forces"]).max() <= 2.5e-6   # grid k-sum (default W = 13)
    assert abs(e - ref["energy"]) <= 1e-9 * np.abs(ref["terms"]).sum() + 1e-6
    assert np.abs(k.dedq() - ref["dedq"]).max() <= 1e-6 * max(1.0, np.abs(ref["dedq"]).max())


def _run_ranks(overlap, world, system, force, pos, box, skin, steps=3, handover="event"):
    """`world` ranks of an atom decomposition driven on one GPU through the split-phase calls
    (cf_compute_begin / direct / end), the all-reduce of B(n) done by hand on the caller's
    stream between begin and end, as openmmcoul.distributed does with RCCL."""
    from openmmcoul.distributed import device_buffer_as_tensor
    stream = torch.cuda.current_stream().cuda_stream
    ks = [HipCalcCoulForceKernel(stream=stream, rank=r, world_size=world, kspace_algo=2,
                                 handover=handover).initialize(system, force) for r in range(world)]
    for k in ks:
        k.set_overlap(overlap)
        if skin:
            k.set_neighbor_skin(skin)
    rng = np.random.default_rng(5)
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    out = []
    for s in range(steps):
        forces = s != 1   # an energy-only evaluation in between
        for k in ks:
            k.begin(pt, box, forces, True)
        bufs = [device_buffer_as_tensor(*k.kspace_buffer(), "cuda") for k in ks]
        total = sum(bufs[1:], bufs[0].clone())
        for b in bufs:
            b.copy_(total)
        f = torch.zeros_like(pt)
        es = []
        for k in ks:
            e = torch.zeros(1, dtype=torch.float64, device="cuda")
            k.end(f if forces else None, e)
            es.append(e)
        torch.cuda.synchronize()
        out.append(([x.item() for x in es], f.cpu().numpy(),
                    [k.dedq()[slice(*k.owned_range())] for k in ks] if forces else None))   # owned atoms
        pt += torch.tensor(rng.normal(scale=0.004, size=pos.shape), device="cuda")
    for k in ks:
        k.destroy()
    return out


@pytest.mark.parametrize("world,skin,handover", [(2, 0.0, "event"), (4, 0.1, "event"), (2, 0.1, "memory")])
def test_multi_rank_overlap_is_bitwise_one_stream(world, skin, handover):
    """Multi-rank split-phase calls: the direct chain on the second stream from cf_compute_begin
    on (cf_api.hip launch_begin_split / launch_end_split) against one stream, bitwise."""
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    a = _run_ranks(True, world, system, force, pos, box, skin, handover=handover)
    b = _run_ranks(False, world, system, force, pos, box, skin)
    for (ea, fa, da), (eb, fb, db) in zip(a, b):
        assert ea == eb and np.array_equal(fa, fb)
        assert (da is None and db is None) or all(np.array_equal(x, y) for x, y in zip(da, db))


def test_set_overlap_at_run_time_is_bitwise():
    """cf_set_overlap switches the second stream off and on between evaluations of one handle
    (the bench's breakdown pass runs one-stream): the same bits every time."""
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    stream = torch.cuda.current_stream().cuda_stream
    k = HipCalcCoulForceKernel(stream=stream, kspace_algo=2).initialize(system, force)
    k.set_neighbor_skin(0.1)
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    res = []
    for on in (True, False, True, False):
        k.set_overlap(on)
        f = torch.zeros_like(pt)
        e = torch.zeros(1, dtype=torch.float64, device="cuda")
        k.execute_device(pt, box, True, True, f, e)
        torch.cuda.synchronize()
        res.append((e.item(), f.cpu().numpy(), k.dedq()))
    k.destroy()
    for e, f, d in res[1:]:
        assert e == res[0][0] and np.array_equal(f, res[0][1]) and np.array_equal(d, res[0][2])


def test_successive_handles_hand_over_from_zero():
    """The memory hand-over's fork / join counters of a new handle start from zero even when its
    allocation reuses a destroyed handle's counters (cf_api.hip ensure_aux): otherwise the old
    counts satisfy the new handle's first waits at once and the second stream starts before its
    producer.  Each of several handles, created after the previous one ran and was destroyed,
    gives on its first evaluations the one-stream bits."""
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    ref = _run(False, system, force, pos, box, 0.0, steps=2)
    for _ in range(4):
        got = _run(True, system, force, pos, box, 0.0, steps=2, handover="memory")
        for (ea, fa, da, ta), (eb, fb, db, tb) in zip(ref, got):
            assert ea == eb and np.array_equal(fa, fb) and np.array_equal(ta, tb)
            if da is not None:
                assert np.array_equal(da, db)


def test_handover_option_validation():
    system, force, pos, box = ts.water_box(100, cutoff=0.6)
    from openmmcoul import ChargeFluxError
    with pytest.raises(ValueError):
        HipCalcCoulForceKernel(kspace_algo=2, handover="spin")
    k = HipCalcCoulForceKernel(kspace_algo=2)
    k._handover = 7   # an out-of-range cf_options.handover reaches cf_create
    with pytest.raises(ChargeFluxError):
        k.initialize(system, force)
