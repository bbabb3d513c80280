"""hipGraph replay of single-rank evaluations (cf_set_graph): the captured launches must give
the same bits as eager calls -- over a trajectory with a kept neighbour list (rebuilds decided
on the device inside the graph), after a box change (re-capture) and with other output buffers
(re-capture) -- and the cache must actually replay.  Bar: bitwise equality."""

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


def _traj(k, pos, box, steps, f=None, e=None, box2=None):
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    f = torch.zeros_like(pt) if f is None else f
    e = torch.zeros(1, dtype=torch.float64, device="cuda") if e is None else e
    rng = np.random.default_rng(4)
    out = []
    for s in range(steps):
        f.zero_()
        k.execute_device(pt, box2 if (box2 is not None and s >= steps // 2) else box, True, True, f, e)
        torch.cuda.synchronize()
        out.append((e.item(), f.cpu().numpy().copy()))
        pt += torch.tensor(rng.normal(scale=0.006, size=pos.shape), device="cuda")
    return out


@pytest.mark.parametrize("algo,precision,skin", [(2, "double", 0.1), (0, "double", 0.0), (2, "mixed", 0.15)])
def test_graph_replay_is_bitwise_eager(algo, precision, skin):
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    stream = torch.cuda.current_stream().cuda_stream
    mk = lambda: HipCalcCoulForceKernel(stream=stream, kspace_algo=algo, precision=precision).initialize(system, force)
    eager, graph = mk(), mk()
    if skin:
        eager.set_neighbor_skin(skin)
        graph.set_neighbor_skin(skin)
    graph.set_graph(True)
    bigger = box * 1.01
    a = _traj(eager, pos, box, 8, box2=bigger)
    b = _traj(graph, pos, box, 8, box2=bigger)
    for (ea, fa), (eb, fb) in zip(a, b):
        assert ea == eb and np.array_equal(fa, fb)
    caps, reps = graph.graph_stats()
    # graphs per evaluation: one, or with the grid k-space on two streams 2 with the event
    # hand-overs (cf_api.hip launch_full: the direct chain and the reciprocal chain; the prologue's
    # two kernels run eagerly since round 6)
    segs = 2 if algo == 2 else 1
    assert reps >= 4 * segs and caps <= 4 * segs, (caps, reps)
    assert eager.neighbor_stats() == graph.neighbor_stats()


def test_graph_recaptures_for_new_buffers_and_flags():
    system, force, pos, box = ts.make("C2")
    stream = torch.cuda.current_stream().cuda_stream
    k = HipCalcCoulForceKernel(stream=stream, kspace_algo=2).initialize(system, force).set_graph(True)
    ref = HipCalcCoulForceKernel(stream=stream, kspace_algo=2).initialize(system, force)
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    e0, f0 = ref.execute_host(pos, box)
    for _ in range(2):
        for buf in range(2):
            f = torch.zeros_like(pt)
            e = torch.zeros(1, dtype=torch.float64, device="cuda")
            k.execute_device(pt, box, True, True, f, e)
            torch.cuda.synchronize()
            assert e.item() == e0 and np.array_equal(f.cpu().numpy(), f0)
        e = torch.zeros(1, dtype=torch.float64, device="cuda")
        k.execute_device(pt, box, False, True, None, e)   # energy only: another graph
        torch.cuda.synchronize()
        assert e.item() == pytest.approx(e0, rel=1e-12, abs=1e-9)
    caps, reps = k.graph_stats()
    assert caps >= 3
    # timing on: eager, same answer
    k.set_timing(True)
    f = torch.zeros_like(pt)
    k.execute_device(pt, box, True, True, f, None)
    torch.cuda.synchronize()
    assert np.array_equal(f.cpu().numpy(), f0)
    assert k.graph_stats()[0] == caps


@pytest.mark.parametrize("case", ["C2", "w4k"])
def test_graph_recapture_sequence_keeps_guards_clear(case):
    """Regression for the round-5 illegal memory access (r5z, first attempt, inside
    test_graph_recaptures_for_new_buffers_and_flags): the same call sequence -- graph mode, fresh
    output buffers every call, an energy-only evaluation between force evaluations (each flag set
    its own capture, so every segment re-captures in turn), then timing on (eager) -- repeated on
    fresh handles, on C2 (per-atom full list) and on a 12k-atom box (cluster-pair list), with the
    device index guards on.  Every call must give the eager handle's bits and no guard may trip
    (cf_get_device_errors == 0): an index outside its buffer would be skipped and reported here
    instead of faulting."""
    if case == "C2":
        system, force, pos, box = ts.make("C2")
    else:
        system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    stream = torch.cuda.current_stream().cuda_stream
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    ref = HipCalcCoulForceKernel(stream=stream, kspace_algo=2).initialize(system, force)
    e0, f0 = ref.execute_host(pos, box)
    for rep in range(3):
        k = HipCalcCoulForceKernel(stream=stream, kspace_algo=2).initialize(system, force).set_graph(True)
        for _ in range(3):
            for buf in range(2):
                f = torch.zeros_like(pt)
                e = torch.zeros(1, dtype=torch.float64, device="cuda")
                k.execute_device(pt, box, True, True, f, e)
                torch.cuda.synchronize()
                assert e.item() == e0 and np.array_equal(f.cpu().numpy(), f0), (rep, buf)
            e = torch.zeros(1, dtype=torch.float64, device="cuda")
            k.execute_device(pt, box, False, True, None, e)
            torch.cuda.synchronize()
            assert e.item() == pytest.approx(e0, rel=1e-12, abs=1e-9)
        k.set_timing(True)
        f = torch.zeros_like(pt)
        k.execute_device(pt, box, True, True, f, None)
        torch.cuda.synchronize()
        assert np.array_equal(f.cpu().numpy(), f0)
        assert k.device_errors() == 0
        k.destroy()
    assert ref.device_errors() == 0


@pytest.mark.parametrize("world", [2, 4])
def test_graph_segments_of_a_decomposed_step_are_bitwise_eager(world):
    """Multi-rank split calls (begin / direct / end) replayed as three graphs per rank, with the
    k-space buffers summed between begin and end (the all-reduce, by hand on one GPU)."""
    from openmmcoul.distributed import device_buffer_as_tensor
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    stream = torch.cuda.current_stream().cuda_stream
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")

    def run(graph):
        ks = [HipCalcCoulForceKernel(stream=stream, rank=r, world_size=world, kspace_algo=2).initialize(system, force)
              for r in range(world)]
        for k in ks:
            k.set_neighbor_skin(0.1)
            if graph:
                k.set_graph(True)
        bufs = [device_buffer_as_tensor(*k.kspace_buffer(), "cuda") for k in ks]
        f = torch.zeros_like(pt)
        es = [torch.zeros(1, dtype=torch.float64, device="cuda") for _ in ks]
        x = pt.clone()
        rng = np.random.default_rng(8)
        out = []
        for s in range(6):
            f.zero_()
            b_s = box if s < 3 else box * 1.01   # the box changes partway (every segment must re-capture)
            for k in ks:
                k.begin(x, b_s, True, True)
            total = sum(bufs[1:], bufs[0].clone())
            for b in bufs:
                b.copy_(total)
            for k in ks:
                k.direct()
            for k, e in zip(ks, es):
                k.end(f, e)
            torch.cuda.synchronize()
            out.append((sum(e.item() for e in es), f.cpu().numpy().copy()))
            x += torch.tensor(rng.normal(scale=0.006, size=pos.shape), device="cuda")
        stats = [k.graph_stats() for k in ks]
        for k in ks:
            k.destroy()
        return out, stats

    a, _ = run(False)
    b, stats = run(True)
    for (ea, fa), (eb, fb) in zip(a, b):
        assert ea == eb and np.array_equal(fa, fb)
    assert all(reps > 0 for _, reps in stats), stats


def test_graph_recaptures_after_list_reallocation():
    # a larger skin grows the neighbour-list buffer (alloc_nlist): launches captured before it
    # point at the freed buffer, so the cache must re-capture (Handle::alloc_epoch in the key)
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4)
    stream = torch.cuda.current_stream().cuda_stream
    mk = lambda: HipCalcCoulForceKernel(stream=stream, kspace_algo=2).initialize(system, force)
    eager, graph = mk(), mk()
    graph.set_graph(True)
    for k in (eager, graph):
        k.set_neighbor_skin(0.05)
    a = _traj(eager, pos, box, 3)
    b = _traj(graph, pos, box, 3)
    caps0, _ = graph.graph_stats()
    for k in (eager, graph):
        k.set_neighbor_skin(0.3)   # capacity grows: nl reallocated
    a += _traj(eager, pos, box, 3)
    b += _traj(graph, pos, box, 3)
    for (ea, fa), (eb, fb) in zip(a, b):
        assert ea == eb and np.array_equal(fa, fb)
    caps1, reps = graph.graph_stats()
    assert caps1 > caps0 and reps >= 2, (caps0, caps1, reps)


def test_graph_recaptures_after_parameter_update():
    """cf_update_parameters changes launch arguments baked into captured graphs (the number of LJ
    types staged in LDS, or no types at all): the next call must re-capture, not replay."""
    from tests.test_gpu_update import _perturb
    system, force, pos, box = ts.water_box(2000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    stream = torch.cuda.current_stream().cuda_stream
    mk = lambda: HipCalcCoulForceKernel(stream=stream, kspace_algo=2).initialize(system, force)
    eager, graph = mk(), mk()
    for k in (eager, graph):
        k.set_neighbor_skin(0.1)
    graph.set_graph(True)
    a = _traj(eager, pos, box, 3)
    b = _traj(graph, pos, box, 3)
    for distinct in (False, True):   # new LJ parameters; then > 64 LJ types (per-atom LJ gathers)
        _perturb(force, np.random.default_rng(5), distinct)
        for k in (eager, graph):
            k.copyParametersToContext(force)
        a += _traj(eager, pos, box, 3)
        b += _traj(graph, pos, box, 3)
    for (ea, fa), (eb, fb) in zip(a, b):
        assert ea == eb and np.array_equal(fa, fb)


def test_graph_replay_restores_reciprocal_dedq_split():
    """A replayed forces graph leaves the reciprocal dE/dq in its own buffer (two streams): the
    handle must know that after replaying it behind an energy-only capture (cf_get_dedq)."""
    system, force, pos, box = ts.make("C2")
    stream = torch.cuda.current_stream().cuda_stream
    k = HipCalcCoulForceKernel(stream=stream, kspace_algo=2).initialize(system, force).set_graph(True)
    ref = HipCalcCoulForceKernel(stream=stream, kspace_algo=2).initialize(system, force)
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    ref.execute_host(pos, box)
    dq_ref = ref.dedq()
    f = torch.zeros_like(pt)
    e = torch.zeros(1, dtype=torch.float64, device="cuda")
    k.execute_device(pt, box, True, True, f, e)    # capture: forces
    k.execute_device(pt, box, False, True, None, e)  # capture: energy only
    k.execute_device(pt, box, True, True, f, e)    # capture: forces
    k.execute_device(pt, box, True, True, f, e)    # replay: forces
    torch.cuda.synchronize()
    assert k.graph_stats()[1] >= 1
    assert np.array_equal(k.dedq(), dq_ref)


def test_graph_flag_alternation_without_host_syncs():
    """The shape of test_graph_replay_restores_reciprocal_dedq_split, where the round-6 session r6c
    saw an illegal memory access: graph mode on C2 (no skin), forces / energy-only / forces captures
    and a replay queued back to back with no host synchronisation between the calls, repeated on
    fresh handles.  Since round 6 every data-dependent index of the C2 kernels is guarded (cell and
    grid-bin bounds that do not add up to the atoms become empty cells / bins, list entries past N,
    a clear rebuild flag without a skin): a broken invariant shows as CF_GUARD_* bits here, and the
    results must be the eager handle's bits."""
    from openmmcoul import _cabi
    system, force, pos, box = ts.make("C2")
    stream = torch.cuda.current_stream().cuda_stream
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    ref = HipCalcCoulForceKernel(stream=stream, kspace_algo=2).initialize(system, force)
    e0, f0 = ref.execute_host(pos, box)
    for rep in range(8):
        k = HipCalcCoulForceKernel(stream=stream, kspace_algo=2).initialize(system, force).set_graph(True)
        fs = [torch.zeros_like(pt) for _ in range(3)]
        es = [torch.zeros(1, dtype=torch.float64, device="cuda") for _ in range(4)]
        k.execute_device(pt, box, True, True, fs[0], es[0])
        k.execute_device(pt, box, False, True, None, es[1])
        k.execute_device(pt, box, True, True, fs[1], es[2])
        k.execute_device(pt, box, True, True, fs[2], es[3])
        torch.cuda.synchronize()
        bits = k.device_errors()
        assert bits == 0, (rep, bits)
        for f in fs:
            assert np.array_equal(f.cpu().numpy(), f0), rep
        assert [e.item() for e in es[:1] + es[2:]] == [e0, e0, e0], rep
        assert es[1].item() == pytest.approx(e0, rel=1e-12, abs=1e-9)
        k.destroy()
    assert ref.device_errors() == 0


@pytest.mark.parametrize("case", ["C2", "w4k"])
def test_graph_two_stream_order_under_changing_flags(case):
    """Fork / join order of the two-stream evaluation (event hand-overs) when graph segments are
    replayed and re-captured in turn: positions move every call (a segment running on stale
    charges, cells or lists would show in the bits), the flags alternate (forces + energy, energy
    only, forces only: each a capture of its own) and some calls get fresh output buffers.  The
    graph handle must give the eager handle's bits at every call, and with no skin the list must
    be rebuilt at every evaluation (a direct chain that read the rebuild flag after the join
    cleared it would skip its build)."""
    if case == "C2":
        system, force, pos, box = ts.make("C2")
    else:
        system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    stream = torch.cuda.current_stream().cuda_stream
    mk = lambda: HipCalcCoulForceKernel(stream=stream, kspace_algo=2).initialize(system, force)
    eager, graph = mk(), mk()
    graph.set_graph(True)
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    rng = np.random.default_rng(12)
    flag_cycle = [(True, True), (False, True), (True, True), (True, False), (True, True)]
    f_keep = torch.zeros_like(pt)
    n = 30
    for s in range(n):
        fl, en = flag_cycle[s % len(flag_cycle)]
        out = []
        for k in (eager, graph):
            f = torch.zeros_like(pt) if s % 3 == 0 else f_keep.zero_().clone()
            e = torch.zeros(1, dtype=torch.float64, device="cuda")
            k.execute_device(pt, box, fl, en, f if fl else None, e if en else None)
            torch.cuda.synchronize()
            out.append((e.item(), f.cpu().numpy().copy()))
        (ea, fa), (eb, fb) = out
        assert ea == eb and np.array_equal(fa, fb), (s, fl, en)
        pt += torch.tensor(rng.normal(scale=0.004, size=pos.shape), device="cuda")
    assert eager.neighbor_stats() == graph.neighbor_stats() == (n, n), (eager.neighbor_stats(), graph.neighbor_stats())
    caps, reps = graph.graph_stats()
    assert reps > 0 and caps > 0, (caps, reps)
