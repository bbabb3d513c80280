"""The benchmark's fused MD harness kernels (csrc/md_harness.hip, not part of the
CoulForce path) against a plain torch fp64 restatement: velocity-Verlet kick/drift for
the owned atoms and the flexible-water harmonic restraints.  Tolerance 1e-12 relative."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

import bench  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _restraints_ref(x, nw):
    f = torch.zeros_like(x)
    w = x[: 3 * nw].view(nw, 3, 3)
    fw = f[: 3 * nw].view(nw, 3, 3)
    for a, b, k, r0 in ((0, 1, bench.K_OH, bench.R_OH0), (0, 2, bench.K_OH, bench.R_OH0),
                        (1, 2, bench.K_HH, bench.R_HH0)):
        d = w[:, b] - w[:, a]
        r = d.norm(dim=1, keepdim=True)
        g = (k * (r - r0) / r) * d
        fw[:, a] += g
        fw[:, b] -= g
    return f


@pytest.mark.parametrize("lo,hi", [(0, 905), (300, 609)])
def test_md_harness_matches_torch(lo, hi):
    rng = np.random.default_rng(5)
    n, nw, dt = 905, 300, 0.001   # 300 waters + 5 ions; owned slice [lo, hi)
    dev = torch.device("cuda", 0)
    o = rng.uniform(0, 3, size=(nw, 3))
    x = np.concatenate([(o[:, None, :] + rng.normal(scale=0.06, size=(nw, 3, 3))).reshape(-1, 3),
                        rng.uniform(0, 3, size=(n - 3 * nw, 3))])
    x = torch.tensor(x, device=dev)
    v = torch.tensor(rng.normal(size=(n, 3)), device=dev)
    f = torch.tensor(rng.normal(size=(n, 3)) * 100, device=dev)
    inv_m = torch.tensor(1.0 / rng.uniform(1, 16, size=(n, 1)), device=dev)
    md = bench.MDHarness(nw, lo, hi, dt, inv_m, torch.cuda.current_stream().cuda_stream)
    own = torch.zeros(n, 1, dtype=torch.float64, device=dev)
    own[lo:hi] = 1
    # kick + drift
    xr, vr = x.clone(), v + 0.5 * dt * f * inv_m * own
    xr = xr + dt * vr * own
    f_before = f.clone()
    md.kick_drift(x, v, f)
    torch.cuda.synchronize()
    assert torch.allclose(v, vr, rtol=1e-12, atol=0) and torch.allclose(x, xr, rtol=1e-12, atol=0)
    # the owned forces are zeroed for the next evaluation to add into; the rest untouched
    assert torch.count_nonzero(f[lo:hi]) == 0
    assert torch.equal(f[:lo], f_before[:lo]) and torch.equal(f[hi:], f_before[hi:])
    # restraints + kick
    fr = f + _restraints_ref(x, nw) * own
    vr = v + 0.5 * dt * fr * inv_m * own
    md.restrain_kick(x, v, f)
    torch.cuda.synchronize()
    assert torch.allclose(f[lo:hi], fr[lo:hi], rtol=1e-12, atol=1e-9)
    assert torch.allclose(v, vr, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("lo,hi,first", [(0, 905, False), (300, 609, False), (0, 905, True)])
def test_md_fused_step_matches_two_kernels(lo, hi, first):
    # md_restrain_kick_drift (the bench's one launch per step) = restrain_kick then kick_drift
    # (without the restraint kick on the first step)
    rng = np.random.default_rng(7)
    n, nw, dt = 905, 300, 0.001
    dev = torch.device("cuda", 0)
    o = rng.uniform(0, 3, size=(nw, 3))
    x0 = np.concatenate([(o[:, None, :] + rng.normal(scale=0.06, size=(nw, 3, 3))).reshape(-1, 3),
                         rng.uniform(0, 3, size=(n - 3 * nw, 3))])
    v0 = rng.normal(size=(n, 3))
    f0 = rng.normal(size=(n, 3)) * 100
    inv_m = torch.tensor(1.0 / rng.uniform(1, 16, size=(n, 1)), device=dev)
    md = bench.MDHarness(nw, lo, hi, dt, inv_m, torch.cuda.current_stream().cuda_stream)
    xa, va, fa = (torch.tensor(a, device=dev) for a in (x0, v0, f0))
    md.restrain_kick(xa, va, fa, kick=not first)
    md.kick_drift(xa, va, fa)
    xb, vb, fb = (torch.tensor(a, device=dev) for a in (x0, v0, f0))
    md.restrain_kick_drift(xb, vb, fb, first)
    torch.cuda.synchronize()
    assert torch.allclose(xb, xa, rtol=1e-14, atol=1e-15)
    assert torch.allclose(vb, va, rtol=1e-13, atol=1e-13)
    assert torch.equal(fb, fa)   # owned rows zeroed, the rest untouched
