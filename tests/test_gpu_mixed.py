"""Mixed precision (CF_PRECISION_MIXED) and the narrow grid kernel it defaults
to (W = 8, spread with 2 source bins per axis).

Accuracy bar: RMS relative force error <= 1e-4 against the fp64 build,
  rms_rel = sqrt(mean |F - F_ref|^2) / sqrt(mean |F_ref|^2);
energies are checked against the magnitude of the terms they are summed from,
  |E - E_ref| <= 1e-7 * (|E_self| + |E_recip| + |E_direct| + |E_excl|),
because the total is a near-cancellation (at C3: self -7.6e6, exclusion +7.5e6, total ~ -1e3
kJ/mol), so a relative bar on the total would measure the cancellation, not the arithmetic.  Charges (flux, fp64 in every mode) stay
exact to 1e-12.  The fp64 reference is the oracle (small systems) or the fp64 HIP path at
the exact k-sum (C3 size)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import Oracle  # noqa: E402
from openmmcoul import HipCalcCoulForceKernel, ChargeFluxError  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402
from openmmcoul.distributed import ShardedCoulKernel  # noqa: E402

GRID = HipCalcCoulForceKernel.KSPACE_GRID
RMS_TOL = 1e-4
E_TOL = 1e-7


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def rms_rel(f, ref):
    return float(np.sqrt(np.mean(np.sum((f - ref) ** 2, axis=1)) / np.mean(np.sum(ref ** 2, axis=1))))


@pytest.mark.parametrize("algo", [0, GRID])
@pytest.mark.parametrize("nw,rc,tol", [(400, 0.7, 1e-4), (1000, 1.0, 1e-3)])
def test_mixed_vs_oracle(algo, nw, rc, tol):
    system, force, pos, box = ts.water_box(nw, cutoff=rc, ewald_tol=tol, every_bond_angle=10)
    k = HipCalcCoulForceKernel(kspace_algo=algo, precision="mixed").initialize(system, force)
    ref = Oracle(force, box).execute(pos, box)
    e, f = k.execute_host(pos, box)
    err = rms_rel(f, ref["forces"])
    print(f"mixed algo {algo} N={3 * nw}: rms_rel {err:.2e}  dE/E {(e - ref['energy']) / ref['energy']:.2e}")
    assert err <= RMS_TOL
    assert abs(e - ref["energy"]) <= E_TOL * np.abs(ref["terms"]).sum()
    assert np.abs(k.charges() - ref["charges"]).max() <= 1e-12
    # the pair kernel alone (exact k-sum) is far inside the bar
    if algo == 0:
        assert err <= 1e-5


def test_mixed_energy_flags_and_skin():
    system, force, pos, box = ts.water_box(400, cutoff=0.7, ewald_tol=1e-4, every_bond_angle=3)
    k = HipCalcCoulForceKernel(kspace_algo=GRID, precision="mixed").initialize(system, force)
    k.set_neighbor_skin(0.1)
    o = Oracle(force, box)
    rng = np.random.default_rng(7)
    p = pos.copy()
    for step in range(6):   # kept and rebuilt lists
        p = p + rng.normal(scale=0.01, size=p.shape)
        for fl, en in ((True, True), (False, True)):
            ref = o.execute(p, box, fl, en)
            e, f = k.execute_host(p, box, fl, en)
            assert abs(e - ref["energy"]) <= E_TOL * np.abs(ref["terms"]).sum()
            if fl:
                assert rms_rel(f, ref["forces"]) <= RMS_TOL


def test_bad_precision_rejected():
    with pytest.raises(ValueError):
        HipCalcCoulForceKernel(precision="half")


@pytest.mark.parametrize("W", [6, 8, 9])
def test_narrow_grid_kernel_fp64(W):
    # fp64 pair kernel, W <= 9 grid (2 source bins per axis in the spread): only the grid
    # truncation error remains, measured against the oracle's exact k-sum
    system, force, pos, box = ts.make("C2")
    k = HipCalcCoulForceKernel(kspace_algo=GRID, grid_width=W).initialize(system, force)
    ref = Oracle(force, box).execute(pos, box)
    e, f = k.execute_host(pos, box)
    err = rms_rel(f, ref["forces"])
    dmax = np.abs(f - ref["forces"]).max()
    print(f"W={W}: rms_rel {err:.2e} max|dF| {dmax:.2e} dE {e - ref['energy']:.2e}")
    assert err <= {6: 1e-4, 8: 1e-5, 9: 3e-6}[W]


def test_mixed_c3_vs_fp64_exact():
    # C3 size: mixed (fp32 pairs, W = 8 grid) against the fp64 exact-k-sum HIP path
    system, force, pos, box = ts.make("C3")
    dev = torch.device("cuda", 0)
    x = torch.tensor(pos, dtype=torch.float64, device=dev)
    out = {}
    for name, kw in (("ref", dict(kspace_algo=0)), ("mixed", dict(kspace_algo=GRID, precision="mixed"))):
        kern = ShardedCoulKernel(system, force, 0, neighbor_skin=0.1, **kw)
        f = torch.zeros_like(x)
        e = kern.execute(x, box, f, include_energy=True)
        torch.cuda.synchronize()
        out[name] = (e.item(), f.cpu().numpy(), kern.kernel.energy_terms())
        del kern
    err = rms_rel(out["mixed"][1], out["ref"][1])
    de = out["mixed"][0] - out["ref"][0]
    print(f"C3 mixed vs fp64: rms_rel {err:.2e} dE {de:.3e} of sum|terms| {np.abs(out['ref'][2]).sum():.3e}")
    assert err <= RMS_TOL
    assert abs(de) <= E_TOL * np.abs(out["ref"][2]).sum()
