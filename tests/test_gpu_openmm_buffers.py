"""cf_compute_openmm: the evaluation on an OpenMM GPU platform's own buffers -- posq (real4) in the
platform's sorted order with atomIndex, forces added into 64-bit fixed-point planes (2^32 units,
stride paddedNumAtoms) and the energy added into an energy-buffer element -- the conventions the
reference's CUDA platform binds its kernels to (platforms/cuda/src/CudaCoulKernels.cpp:523-600).

Buffers are built from the synthetic systems with a shuffled atomIndex (OpenMM reorders atoms
spatially) and pre-filled force / energy contents, and checked against the oracle:
  forces  max |dF| <= 1e-8 kJ/mol/nm (exact k-sum) / 2.5e-6 (grid k-sum), after the fixed-point
          conversion (resolution 2^-32 = 2.3e-10)
  energy  |dE| <= 1e-9 |E| + 1e-8 kJ/mol
posq is never written (the reference's CUDA platform overwrites posq.w with the flux charges,
SURVEY A.3)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import Oracle  # noqa: E402
from openmmcoul import HipCalcCoulForceKernel, ChargeFluxError, _cabi  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402

FIX = 2.0 ** 32


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _platform_buffers(pos, rng, padded, dtype=torch.float64, with_correction=False):
    """OpenMM-style device buffers: atomIndex = a random permutation, posq[s] = (pos[atomIndex[s]], w)."""
    n = len(pos)
    perm = rng.permutation(n).astype(np.int32)
    w = rng.normal(size=n)   # the platform's own charge slot: must come back untouched
    p = np.concatenate([pos[perm], w[:, None]], axis=1)
    corr = None
    if dtype == torch.float32:
        hi = p.astype(np.float32)
        if with_correction:   # the mixed platform: posq + posqCorrection = the fp64 position
            corr = torch.tensor((p - hi.astype(np.float64)).astype(np.float32), device="cuda")
        posq = torch.tensor(hi, device="cuda")
    else:
        posq = torch.tensor(p, dtype=torch.float64, device="cuda")
    idx = torch.tensor(perm, device="cuda")
    fbuf0 = rng.integers(-2 ** 40, 2 ** 40, size=3 * padded, dtype=np.int64)   # other forces' contributions
    return perm, posq, corr, idx, fbuf0


def _forces_from_buffer(fbuf, fbuf0, perm, padded, n):
    d = (fbuf - fbuf0).reshape(3, padded)[:, :n].astype(np.float64) / FIX   # by sorted slot
    f = np.zeros((n, 3))
    f[perm] = d.T
    return f


@pytest.mark.parametrize("case,algo,f_tol", [("C2", 0, 1e-8), ("C2", 2, 2.5e-6), ("w4k", 2, 2.5e-6)])
def test_openmm_buffers_match_oracle(case, algo, f_tol):
    if case == "C2":
        system, force, pos, box = ts.make("C2")
    else:   # 12k atoms: the cluster-pair list (>= 4 cells per axis)
        system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    ref = Oracle(force, box).execute(pos, box)
    n = len(pos)
    padded = (n + 31) // 32 * 32
    rng = np.random.default_rng(7)
    perm, posq, _, idx, fbuf0 = _platform_buffers(pos, rng, padded)
    posq0 = posq.clone()
    stream = torch.cuda.current_stream().cuda_stream
    k = HipCalcCoulForceKernel(stream=stream, kspace_algo=algo).initialize(system, force)
    fbuf = torch.tensor(fbuf0, device="cuda")
    ebuf = torch.tensor([12.5], dtype=torch.float64, device="cuda")
    k.execute_openmm(posq, idx, padded, box, True, True, fbuf, ebuf)
    torch.cuda.synchronize()
    f = _forces_from_buffer(fbuf.cpu().numpy(), fbuf0, perm, padded, n)
    assert np.abs(f - ref["forces"]).max() <= f_tol, np.abs(f - ref["forces"]).max()
    # padding entries are not touched
    tail = (fbuf.cpu().numpy() - fbuf0).reshape(3, padded)[:, n:]
    assert not tail.any()
    e = ebuf.item() - 12.5
    assert abs(e - ref["energy"]) <= 1e-9 * abs(ref["energy"]) + 1e-8, (e, ref["energy"])
    assert torch.equal(posq, posq0)   # posq (incl. w) is read only
    # the same result through the atom-order entry point, bit for bit
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    f2 = torch.zeros_like(pt)
    e2 = torch.zeros(1, dtype=torch.float64, device="cuda")
    k.execute_device(pt, box, True, True, f2, e2)
    torch.cuda.synchronize()
    f_fix = np.trunc(f2.cpu().numpy() * FIX) / FIX   # OpenMM's conversion truncates toward zero
    assert np.array_equal(f, f_fix)
    assert k.device_errors() == 0


def test_openmm_buffers_mixed_platform_float4_with_correction():
    """float4 posq + posqCorrection (OpenMM's mixed precision): positions rebuilt in fp64 to ~1e-14 nm,
    the fp64 evaluation on them; energy into a float32 element (single precision's buffer type)."""
    system, force, pos, box = ts.make("C2")
    ref = Oracle(force, box).execute(pos, box)
    n = len(pos)
    padded = n + 64
    rng = np.random.default_rng(3)
    perm, posq, corr, idx, fbuf0 = _platform_buffers(pos, rng, padded, torch.float32, with_correction=True)
    k = HipCalcCoulForceKernel(stream=torch.cuda.current_stream().cuda_stream, kspace_algo=0).initialize(system, force)
    fbuf = torch.tensor(fbuf0, device="cuda")
    ebuf = torch.zeros(1, dtype=torch.float32, device="cuda")
    k.execute_openmm(posq, idx, padded, box, True, True, fbuf, ebuf, posq_correction=corr)
    torch.cuda.synchronize()
    f = _forces_from_buffer(fbuf.cpu().numpy(), fbuf0, perm, padded, n)
    assert np.abs(f - ref["forces"]).max() <= 1e-7, np.abs(f - ref["forces"]).max()
    assert abs(ebuf.item() - ref["energy"]) <= 1e-6 * abs(ref["energy"]), (ebuf.item(), ref["energy"])


def test_openmm_buffers_energy_only_and_graph_replay():
    """Energy only leaves the force planes alone; in graph mode repeated calls replay and give the
    eager bits (the gather / scatter run eagerly around the replayed evaluation)."""
    system, force, pos, box = ts.water_box(2000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    n = len(pos)
    padded = (n + 31) // 32 * 32
    rng = np.random.default_rng(11)
    perm, posq, _, idx, fbuf0 = _platform_buffers(pos, rng, padded)
    stream = torch.cuda.current_stream().cuda_stream
    eager = HipCalcCoulForceKernel(stream=stream, kspace_algo=2).initialize(system, force)
    graph = HipCalcCoulForceKernel(stream=stream, kspace_algo=2).initialize(system, force).set_graph(True)
    fb = torch.tensor(fbuf0, device="cuda")
    eb = torch.zeros(1, dtype=torch.float64, device="cuda")
    eager.execute_openmm(posq, idx, padded, box, False, True, fb, eb)
    torch.cuda.synchronize()
    assert np.array_equal(fb.cpu().numpy(), fbuf0) and eb.item() != 0.0
    outs = []
    for k in (eager, graph):
        res = []
        for _ in range(4):
            fb = torch.tensor(fbuf0, device="cuda")
            eb = torch.zeros(1, dtype=torch.float64, device="cuda")
            k.execute_openmm(posq, idx, padded, box, True, True, fb, eb)
            torch.cuda.synchronize()
            res.append((eb.item(), fb.cpu().numpy()))
        outs.append(res)
    for (ea, fa), (eb_, fb_) in zip(*outs):
        assert ea == eb_ and np.array_equal(fa, fb_)
    assert graph.graph_stats()[1] > 0


def test_bad_atom_index_trips_a_guard_not_a_fault():
    """An atomIndex entry outside [0, N) is caller data the kernels cannot trust: the gather skips
    it and sets CF_GUARD_ATOM_INDEX; the handle then fails every later call with CF_ERR_STATE
    (device index guards, include/chargeflux.h) instead of faulting the GPU."""
    system, force, pos, box = ts.make("C2")
    n = len(pos)
    rng = np.random.default_rng(5)
    perm, posq, _, idx, fbuf0 = _platform_buffers(pos, rng, n)
    idx[17] = n + 1000
    k = HipCalcCoulForceKernel(stream=torch.cuda.current_stream().cuda_stream, kspace_algo=2).initialize(system, force)
    fb = torch.tensor(fbuf0, device="cuda")
    k.execute_openmm(posq, idx, n, box, True, True, fb, None)
    torch.cuda.synchronize()
    assert k.device_errors() == _cabi.CF_GUARD_ATOM_INDEX
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    with pytest.raises(ChargeFluxError) as ei:
        k.execute_device(pt, box, True, True, torch.zeros_like(pt), None)
    assert ei.value.code == _cabi.CF_ERR_STATE and "atom_index" in str(ei.value)
    with pytest.raises(ChargeFluxError):
        k.energy_terms()
    # a fresh handle is clean
    k2 = HipCalcCoulForceKernel(stream=torch.cuda.current_stream().cuda_stream, kspace_algo=2).initialize(system, force)
    e, f = k2.execute_host(pos, box)
    assert k2.device_errors() == 0 and np.isfinite(e)
