#!/usr/bin/env python3
"""Benchmark: ns/day + ms/force-eval of the charge-flux CoulForce on a periodic water box.

A step = one velocity-Verlet MD step (dt = 1 fs) of the flexible charge-flux water box:
one full CoulForce evaluation (forces + energy: flux charges, Ewald real space with erfc,
reciprocal k-sum, self term, exclusion correction, dE/dq chain rule) on the GPU through
the C-ABI, plus harmonic O-H/H-H restraints and the integrator update (torch, plumbing).

Single node, one process per GPU:
  python bench.py --gpus 1 --steps 20 --warmup 5
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W
Multi-GPU = atom decomposition of one system (strong scaling): per step one RCCL
all-reduce of the structure factors S(k), one of the energy and one to re-replicate the
integrated positions.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "openmm-chargeflux_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from openmmcoul import testsystems as ts  # noqa: E402
from openmmcoul.distributed import ShardedCoulKernel  # noqa: E402

METRIC = "ns/day + ms/force-eval, periodic charge-flux box, 1/2/4/8 MI355X"
FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (= dense FP64 matrix) peak, vendor spec
FP32_PEAK_TFLOPS = 157.3  # MI355X FP32 vector peak (the mixed-precision pair kernel)
HBM_PEAK_GBS = 8000.0
K_OH, R_OH0 = 345000.0, 0.09572      # harness restraints (kJ/mol/nm^2, nm)
K_HH, R_HH0 = 230000.0, 0.15139
KB = 0.0083144626                     # kJ/mol/K


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class MDHarness:
    """Velocity Verlet + flexible-water restraints as two fused HIP kernels per step
    (libcf_mdharness.so, csrc/md_harness.hip; not part of the CoulForce path)."""

    def __init__(self, n_waters, lo, hi, dt, inv_mass, stream):
        import ctypes as C
        path = os.path.join(ROOT, "openmm-chargeflux_amd", "libcf_mdharness.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run __graft_entry__.build() (make -C openmm-chargeflux_amd/csrc)")
        L = C.CDLL(path)
        vp, d, i = C.c_void_p, C.c_double, C.c_int
        L.md_kick_drift.argtypes = [i, i, d, vp, vp, vp, vp, vp]
        L.md_restrain_kick.argtypes = [i, i, i, d, d, d, d, d, vp, vp, vp, vp, vp]
        L.md_restrain_kick_drift.argtypes = [i, i, i, d, d, d, d, d, i, vp, vp, vp, vp, vp]
        self.L, self.C = L, C
        self.nw, self.lo, self.hi, self.dt = n_waters, lo, hi, dt
        self.inv_m = inv_mass
        self.stream = C.c_void_p(stream)

    def kick_drift(self, pos, vel, frc):   # also zeroes frc[lo:hi] (its last reader in the step)
        rc = self.L.md_kick_drift(self.lo, self.hi, self.dt, pos.data_ptr(), vel.data_ptr(), frc.data_ptr(),
                                  self.inv_m.data_ptr(), self.stream)
        assert rc == 0

    def restrain_kick_drift(self, pos, vel, frc, first):
        # f += restraints ; v += dt/2 f/m (not on the first step) ; v += dt/2 f/m ; x += dt v ; f = 0
        rc = self.L.md_restrain_kick_drift(self.lo, self.hi, self.nw, K_OH, R_OH0, K_HH, R_HH0, self.dt, int(first),
                                           pos.data_ptr(), vel.data_ptr(), frc.data_ptr(), self.inv_m.data_ptr(),
                                           self.stream)
        assert rc == 0

    def restrain_kick(self, pos, vel, frc, kick=True):
        rc = self.L.md_restrain_kick(self.lo, self.hi, self.nw, K_OH, R_OH0, K_HH, R_HH0, self.dt if kick else 0.0,
                                     pos.data_ptr(), vel.data_ptr(), frc.data_ptr(), self.inv_m.data_ptr(), self.stream)
        assert rc == 0


# Calibration of the oracle's serial timing against the compiled reference kernel
# (measured in the survey session on this image's build host): oracle time /
# reference time, measured by tools/calibrate_cpu.py in the same container.
CPU_CALIBRATION = os.path.join(ROOT, "profiles", "cpu_calibration.json")


def host_cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(force, pos, box, k_sample):
    from oracle import Oracle
    o = Oracle(force, box)
    tn, tr, kt = o.time_sample(pos, box, k_sample)
    t_eval = tn + tr * kt / k_sample
    cal = ""
    if os.path.exists(CPU_CALIBRATION):
        c = json.load(open(CPU_CALIBRATION))
        cal = (f"; oracle/compiled-reference time ratio {c['ratio_summary']} measured on the build host "
               f"({c['host']}), tools/calibrate_cpu.py")
    return {
        "value": 0.0864 / t_eval,   # ns/day at dt = 1 fs (t_eval in s), force evaluation only
        "unit": "ns/day",
        "cores": 1,
        "kind": "port",
        "ms_per_force_eval": t_eval * 1e3,
        "host_cpu": host_cpu_model(),
        "k_sample_fraction": round(k_sample / kt, 4),
        "sample": (f"C3 on the oracle (serial fp64 restatement of ReferenceCoulKernels.cpp, same "
                   f"two-pass cos/sin k-loop, O(N) cell list), 1 core of {host_cpu_model()}: full flux/self/"
                   f"real-space/exclusion/chain-rule part ({tn:.2f} s) + first {k_sample} of {kt} reciprocal "
                   f"k-vectors ({100.0 * k_sample / kt:.1f} % of K, {tr:.2f} s), extrapolated linearly in K to "
                   f"{t_eval:.1f} s/eval" + cal),
    }


# rocprofv3 kernel names of the library's timing phases, up to their template arguments (the
# instantiation that runs in the profiled command; a phase timed as one bracket may be several
# launches: their bytes are summed).  The pair kernel follows the list kind (cf_get_pair_list).
PMC_KERNEL = {"kspace_force": ["cf::k_force<"], "kspace_sfac": ["cf::k_sfac<"],
              "grid_spread": ["cf::k_g_spread_mfma<"], "grid_interp": ["cf::k_g_interp2<"]}
PAIR_KERNEL = {"cluster": "cf::k_pairs_cq<", "atom_half": "cf::k_pairs_half<", "full": "cf::k_pairs<"}


def pair_count(force, pos, box):
    """P_c: non-excluded pairs with r <= rc under minimum image (the reference's neighbour
    list, ReferenceCoulKernels.cpp:559), at the initial positions."""
    from scipy.spatial import cKDTree
    L = np.array([box[0][0], box[1][1], box[2][2]])
    rc = force.getCutoffDistance()
    w = np.mod(pos, L)
    w[w >= L] = 0.0
    n_all = (cKDTree(w, boxsize=L).count_neighbors(cKDTree(w, boxsize=L), rc) - len(pos)) // 2
    ex = {tuple(sorted(force.getExceptionParameters(k)[:2])) for k in range(force.getNumExceptions())}
    n_ex = 0
    for a, b in ex:
        d = pos[a] - pos[b]
        d -= L * np.round(d / L)
        n_ex += int(np.dot(d, d) <= rc * rc)
    return int(n_all - n_ex)


def pmc_traffic(config, world, phase, precision, pair_list):
    """HBM bytes per launch of the dominant kernel from the newest committed PMC summary of this
    workload -- profiles/r*_c3_pmc_summary*.json (fp64 C3) or r*_c5_pmc_summary*.json (mixed C5),
    written by tools/profile_round.sh / the session scripts from separate rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of this same bench command, with the gfx950 FETCH_SIZE
    correction -- newest = highest round, a "final" summary first.  None when no profile matches."""
    wl = {("C3", "double"): "c3", ("C5", "mixed"): "c5"}.get((config, precision))
    if wl is None or world != 1:
        return None, None
    import glob
    import re

    def newest(f):
        m = re.match(r"r(\d+)", os.path.basename(f))
        return (int(m.group(1)) if m else -1, "final" in os.path.basename(f), os.path.basename(f))

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{wl}_pmc_summary*.json")), key=newest)
    if not files:
        return None, None
    summary = json.load(open(files[-1]))
    total = 0
    prefixes = [PAIR_KERNEL.get(pair_list, "?")] if phase == "direct_pairs" else PMC_KERNEL[phase]
    if phase == "direct_pairs" and pair_list == "full" and precision == "mixed":
        prefixes = ["cf::k_pairs_mixed<"]
    for prefix in prefixes:
        hits = [e for name, e in summary.items() if isinstance(e, dict) and name.startswith(prefix)
                and "hbm_read_bytes_est" in e and "hbm_write_bytes" in e]
        if len(hits) != 1:   # none, or several instantiations profiled: no unambiguous figure
            return None, None
        total += hits[0]["hbm_read_bytes_est"] + hits[0]["hbm_write_bytes"]
    return int(total), os.path.relpath(files[-1], ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="C3", choices=["C2", "C3", "C5"])
    ap.add_argument("--kspace-algo", type=int, default=2,
                    help="0 exact k-sum (fp64 MFMA), 1 exact (direct VALU), 2 grid (ES spread / pruned DFT)")
    ap.add_argument("--grid-width", type=int, default=0,
                    help="ES kernel width for --kspace-algo 2 (0 = 14, or 8 with --precision mixed)")
    ap.add_argument("--precision", default="double", choices=["double", "mixed"],
                    help="mixed: fp32 direct-space pair kernel (fp32 force / fp64 energy accumulation), W=8 grid")
    ap.add_argument("--no-exact-compare", action="store_true",
                    help="skip timing the exact k-sum path beside the grid path")
    ap.add_argument("--cpu-k-sample", type=int, default=0,
                    help="k-vectors of the CPU-baseline sample (0 = 10%% of K_half)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="no per-kernel HIP events in the timed steps (measures their overhead; no roofline)")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: replay each step's CoulForce launches as a captured hipGraph (cf_set_graph) in the "
                         "timed region")
    ap.add_argument("--pair-list", default="auto", choices=["auto", "cluster", "atom_half", "full"],
                    help="direct-space list (cf_options.pair_list; auto: the 18-cell cluster-pair list on one fp64 rank)")
    ap.add_argument("--handover", default="event", choices=["event", "memory"],
                    help="fork / join of the library's second stream (cf_options.handover; memory: opt-in)")
    ap.add_argument("--variants", type=lambda v: int(v, 0), default=0,
                    help="cf_options.variants bits (A/B kernels of the same sums; include/chargeflux.h)")
    ap.add_argument("--dt", type=float, default=0.001, help="ps")
    ap.add_argument("--neighbor-skin", type=float, default=None,
                    help="nm; persistent list rebuilt when an atom moved > skin/2 (0 = every step); default "
                         "0.125 (C3), 0.15 (C2) or 0.2 (C5): the optima of the cluster-pair list's re-sweep, "
                         "profiles/r05an_skin_resweep.txt (round 2's per-atom lists: r02_skin_sweep_m.txt)")
    args = ap.parse_args()
    if args.neighbor_skin is None:
        args.neighbor_skin = {"C5": 0.2, "C3": 0.125}.get(args.config, 0.15)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the multi-rank path on a one-GPU box (not a benchmark configuration):
    # CF_BENCH_ONE_GPU=1 puts every rank on device 0, CF_BENCH_BACKEND=gloo replaces RCCL
    if os.environ.get("CF_BENCH_ONE_GPU") == "1":
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("CF_BENCH_BACKEND", "nccl")
        dist.init_process_group(backend, **({"device_id": dev} if backend == "nccl" else {}))

    t_setup = time.time()
    system, force, pos_np, box = ts.make(args.config)
    n = len(pos_np)
    n_waters = force.getNumFluxWaters() + force.getNumFluxAngles()
    kern = ShardedCoulKernel(system, force, local, kspace_algo=args.kspace_algo, neighbor_skin=args.neighbor_skin,
                             grid_width=args.grid_width, precision=args.precision, handover=args.handover,
                             pair_list=args.pair_list, variants=args.variants)
    lo, hi = kern.lo, kern.hi
    alpha, kmax = kern.kernel.ewald_params()
    k_half = (kmax[2] - 1) + (kmax[1] - 1) * (2 * kmax[2] - 1) + (kmax[0] - 1) * (2 * kmax[1] - 1) * (2 * kmax[2] - 1)

    pos = torch.tensor(pos_np, dtype=torch.float64, device=dev)
    masses = torch.tensor([system._masses[i] for i in range(n)], dtype=torch.float64, device=dev).view(-1, 1)
    rng = np.random.default_rng(ts.SEED + 1)
    v0 = rng.normal(size=(n, 3)) * np.sqrt(KB * 300.0 / masses.cpu().numpy())
    vel = torch.tensor(v0, dtype=torch.float64, device=dev)
    frc = torch.zeros_like(pos)
    dt = args.dt
    log(f"[rank {rank}] setup {time.time() - t_setup:.1f}s  N={n} owned=[{lo},{hi}) alpha={alpha:.5f} "
        f"kmax={kmax} K_half={k_half}")

    md = MDHarness(n_waters, lo, hi, dt, (1.0 / masses).contiguous(), torch.cuda.current_stream(dev).cuda_stream)
    frc.zero_()
    energy = kern.execute(pos, box, frc, include_energy=True)
    ev = []
    first = [True]

    def step(record):
        # the previous step's restraints and second half kick fused with this step's first half
        # kick and drift (one harness launch per step; f = 0 afterwards for the force evaluation)
        md.restrain_kick_drift(pos, vel, frc, first[0])
        first[0] = False
        kern.replicate_positions(pos)
        if record:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
        e = kern.execute(pos, box, frc, include_energy=True)   # forces ADDED into the zeroed frc
        if record:
            b.record()
            ev.append((a, b))
        return e

    for _ in range(args.warmup):
        energy = step(False)
    torch.cuda.synchronize()
    # breakdown pass (not the timed region): every phase bracketed by HIP events on the
    # library's stream, with the second stream off (cf_set_overlap) so that each phase's time is
    # its own, not stretched by kernels of the other chain sharing the CUs.  Those event records
    # cost ~10% of a step, so the timed region below brackets only the dominant kernel.
    HOT = ("direct_pairs", "grid_spread", "grid_interp", "kspace_sfac", "kspace_force")
    kern.kernel.set_overlap(False)
    kern.kernel.set_timing(True)
    for _ in range(args.steps):
        energy = step(True)
    torch.cuda.synchronize()
    timing_all = kern.kernel.timing()
    kern.kernel.set_timing(False)
    kern.kernel.set_overlap(True)   # the library's default
    ms_eval = float(np.mean([a.elapsed_time(b) for a, b in ev])) if ev else float("nan")
    per_step = {k: v[0] / args.steps for k, v in timing_all.items()}   # amortized (list phases are not every step)
    dom = max((k for k in HOT if per_step.get(k, 0.0) > 0), key=lambda k: per_step[k], default=None)

    # timed region: K steps, barrier + synchronize on both sides, max over ranks
    if args.graph and world == 1:
        kern.kernel.set_graph(True)   # replayed graphs cannot carry the per-launch events
    elif dom is not None and not args.no_kernel_timing:
        kern.kernel.set_timing(True, phases=[dom])
    builds0, evals0 = kern.kernel.neighbor_stats()
    fb0 = kern.kernel.fallback_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        energy = step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    timing = kern.kernel.timing()
    builds1, evals1 = kern.kernel.neighbor_stats()
    fb1 = kern.kernel.fallback_stats()
    kern.kernel.set_timing(False)
    # force-evaluation pass (after the timed region, not part of it): K more MD steps with two
    # torch events around each execute (the library's stream is torch's current stream) and no
    # library timing at all -> ms_per_force_eval without instrumentation
    ev.clear()
    for _ in range(args.steps):
        energy = step(True)
    torch.cuda.synchronize()
    ms_eval_events = float(np.mean([a.elapsed_time(b) for a, b in ev])) if ev else float("nan")
    # harness pass: K steps of the MD harness alone (restraints, integrator, position all-gather;
    # no CoulForce call), wall clock.  ms_per_force_eval = ms_per_step - this: what the force
    # evaluation adds to a step.  (The event-bracketed figure above reads longer than a whole
    # step at C5 -- 2.82 against 2.69 ms in round 4: two extra event records per step on the
    # library's stream delay the launches they sit between -- so it is reported beside it only.)
    # (the harness alone integrates without fresh forces: positions and velocities are restored
    # after it, or the passes below would start from K steps of free flight -- overlapping
    # molecules, the fp64 rescan fallback on every step: 0.5 -> 4000 ms per step at K = 40)
    saved = (pos.clone(), vel.clone(), frc.clone())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t_h0 = time.perf_counter()
    for _ in range(args.steps):
        md.restrain_kick_drift(pos, vel, frc, False)
        kern.replicate_positions(pos)
    torch.cuda.synchronize()
    ms_harness = (time.perf_counter() - t_h0) / args.steps * 1e3
    pos.copy_(saved[0]); vel.copy_(saved[1]); frc.copy_(saved[2])
    del saved
    # graph pass (after the timed region, not part of it): K steps with the CoulForce launches
    # replayed as a captured hipGraph, wall clock; measures what graph replay would give `value`
    graph_ms = None
    if world == 1 and not args.graph:
        kern.kernel.set_graph(True)
        for _ in range(3):
            energy = step(False)
        torch.cuda.synchronize()
        tg = time.perf_counter()
        for _ in range(args.steps):
            energy = step(False)
        torch.cuda.synchronize()
        graph_ms = (time.perf_counter() - tg) / args.steps * 1e3
        gstats = kern.kernel.graph_stats()
        kern.kernel.set_graph(False)
    kern.synchronize()   # energy all-reduce still in flight (multi-rank)
    e_final = energy.item()
    ms_step = elapsed / args.steps * 1e3
    ms_eval_clean = ms_step - ms_harness
    ns_day = 86.4 / ms_step * (dt / 0.001)

    per_launch = {k: (v[0] / v[1] if v[1] else 0.0) for k, v in timing_all.items()}   # isolated (breakdown pass)
    dom_isolated_ms = per_launch.get(dom) if dom is not None else None
    if dom is not None and timing.get(dom, (0, 0))[1]:
        per_launch[dom] = timing[dom][0] / timing[dom][1]   # measured inside the timed region
    n_own = hi - lo
    # algorithmic work per launch of each hot phase: (HBM bytes,
    # flops, compute pipe, its peak)
    #  direct_pairs  (k_pairs_cq on one fp64 rank, k_pairs_half in mixed precision, k_pairs on
    #                several ranks) bytes 4 P_c + 80 N (a 4-B list entry per pair + per-atom in/out),
    #                flops 80 P_c on the fp64 VALU (fp32 VALU for the mixed-precision kernel); P_c
    #                counts each pair once
    #  grid_spread   2 N W^3 fp64 flops (one FMA per atom x grid point of its support; on the matrix
    #                cores for W > 9, k_g_spread_mfma: the fp64 MFMA and VALU peaks are both 78.6
    #                TF/s), bytes 24 N W (the atom's three tap rows) + 8 ng^3 (grid out)
    #  grid_interp   4 N W^3 fp64 VALU flops (two FMAs per grid value), bytes 8 ng^3 + 24 N W + 32 N
    #  kspace_sfac / kspace_force (exact path)  4 / 8 fp64 MFMA flops per atom x half-space k-vector
    # fraction of the roof = max(B / BW, F / P) / t; "bound" names the larger term
    w_grid = kern.kernel.grid_width() if args.kspace_algo == 2 else 0   # the library's choice (0: its default)
    roofline, others = None, {}
    if dom is not None:
        p_c = pair_count(force, pos_np, box) * n_own / n
        units = float(n_own) * k_half
        ng3 = float(np.prod(kern.kernel.grid_shape())) if args.kspace_algo == 2 else 0.0
        pair_pipe = ("valu", FP64_PEAK_TFLOPS) if args.precision == "double" else ("valu_fp32", FP32_PEAK_TFLOPS)
        alg = {"direct_pairs": (4.0 * p_c + 80.0 * n_own, 80.0 * p_c) + pair_pipe,
               "grid_spread": (24.0 * n_own * w_grid + 8.0 * ng3, 2.0 * n_own * w_grid ** 3,
                               "mfma" if w_grid > 9 else "valu",
                               FP64_PEAK_TFLOPS),
               "grid_interp": (8.0 * ng3 + 24.0 * n_own * w_grid + 32.0 * n_own, 4.0 * n_own * w_grid ** 3, "valu",
                               FP64_PEAK_TFLOPS),
               "kspace_sfac": (64.0 * n_own, 4.0 * units, "mfma", FP64_PEAK_TFLOPS),
               "kspace_force": (64.0 * n_own, 8.0 * units, "mfma", FP64_PEAK_TFLOPS)}

        def roof(k, t_ms):
            b, f, pipe, peak_tf = alg[k]
            t = t_ms * 1e-3
            tb, tf = b / (HBM_PEAK_GBS * 1e9), f / (peak_tf * 1e12)
            return {"bound": "hbm" if tb >= tf else pipe, "frac": max(tb, tf) / t, "gbs": b / t / 1e9,
                    "tflops": f / t / 1e12, "peak_tflops": peak_tf, "alg_bytes": b, "alg_flops": f}

        present = [k for k in alg if per_step.get(k, 0.0) > 0]
        r = roof(dom, per_launch[dom])
        traffic, traffic_src = pmc_traffic(args.config, world, dom, args.precision, kern.kernel.pair_list())
        if r["bound"] == "hbm":
            achieved, peak, unit = r["gbs"], HBM_PEAK_GBS, "GB/s"
        else:
            achieved, peak, unit = r["tflops"], r["peak_tflops"], "TFLOP/s"
        roofline = {"kernel": dom, "bound": r["bound"], "achieved": round(achieved, 3), "peak": peak, "unit": unit,
                    "frac": round(r["frac"], 4), "traffic": traffic, "traffic_source": traffic_src,
                    "traffic_ratio": round(traffic / r["alg_bytes"], 3) if traffic else None,
                    "alg_bytes_per_launch": r["alg_bytes"], "alg_flops_per_launch": r["alg_flops"],
                    "hbm_gbs": round(r["gbs"], 1), "tflops": round(r["tflops"], 3),
                    "avg_launch_ms": per_launch[dom], "pairs_within_cutoff": int(p_c),
                    "frac_definition": "max(alg_bytes/8 TB/s, alg_flops/peak)/t (SURVEY 8(d))"}
        if dom_isolated_ms:
            ri = roof(dom, dom_isolated_ms)
            roofline["isolated"] = {
                "avg_launch_ms": dom_isolated_ms, "frac": round(ri["frac"], 4), "tflops": round(ri["tflops"], 3),
                "hbm_gbs": round(ri["gbs"], 1),
                "note": "the same kernel in the breakdown pass, second stream off (cf_set_overlap): its own "
                        "duration; the timed region's avg_launch_ms includes CUs shared with the reciprocal "
                        "chain running beside it"}
        others = {}
        for k in present:
            if k == dom:
                continue
            rk = roof(k, per_launch[k])
            others[k] = {"avg_launch_ms": round(per_launch[k], 4), "bound": rk["bound"], "frac": round(rk["frac"], 4),
                         "tflops": round(rk["tflops"], 3), "hbm_gbs": round(rk["gbs"], 1)}
    exact = None
    if world == 1 and args.kspace_algo == 2 and not args.no_exact_compare:
        # the exact fp64 k-sum path (kspace_algo 0) timed beside the grid path on the same
        # positions: force evaluations only, HIP events around each
        ke = ShardedCoulKernel(system, force, local, kspace_algo=0, neighbor_skin=args.neighbor_skin)
        fe = torch.zeros_like(pos)
        for _ in range(3):
            ke.execute(pos, box, fe, include_energy=True)
        evs = []
        for _ in range(10):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fe.zero_()
            ee = ke.execute(pos, box, fe, include_energy=True)
            b.record()
            evs.append((a, b))
        fg = torch.zeros_like(pos)
        eg = kern.execute(pos, box, fg, include_energy=True)
        torch.cuda.synchronize()
        d2 = ((fg - fe) ** 2).sum(1).mean().item()
        exact = {"ms_per_force_eval": round(float(np.mean([a.elapsed_time(b) for a, b in evs])), 4),
                 "max_abs_dforce_grid_vs_exact": float((fg - fe).abs().max().item()),
                 "rms_rel_dforce_vs_exact": float(math.sqrt(d2 / (fe ** 2).sum(1).mean().item())),
                 "denergy_grid_vs_exact": float(eg.item() - ee.item())}
        del ke

    host = None
    if world == 1 and not args.no_exact_compare:
        # the host-buffer boundary (cf_compute_host: what a Reference/CPU-platform adapter
        # calls): positions H2D, forces D2H and a stream sync inside every call -- the
        # PCIe-inclusive rate, never `value`
        pos_h = pos.cpu().numpy()
        f_h = np.zeros_like(pos_h)
        for _ in range(3):
            kern.kernel.execute_host(pos_h, box, forces=f_h)
        reps = 20
        t_h = time.perf_counter()
        for _ in range(reps):
            kern.kernel.execute_host(pos_h, box, forces=f_h)
        ms_h = (time.perf_counter() - t_h) / reps * 1e3
        host = {"ms_per_force_eval": round(ms_h, 4), "bytes_h2d": int(pos_h.nbytes), "bytes_d2h": int(f_h.nbytes),
                "note": "cf_compute_host with host positions/forces, wall clock over 20 calls (each syncs); "
                        "compare ms_per_force_eval (device-resident)"}
    openmm_buf = None
    if world == 1 and not args.no_exact_compare:
        # an OpenMM GPU platform's own buffers (cf_compute_openmm: sorted posq + atomIndex in,
        # 2^32 fixed-point force planes and an energy element out; no copies): the device-resident
        # rate through that boundary, events around each call as ms_per_force_eval's pass
        perm = torch.randperm(n, generator=torch.Generator().manual_seed(3)).to(dev)
        posq = torch.cat([pos[perm], torch.zeros(n, 1, dtype=torch.float64, device=dev)], 1).contiguous()
        aidx = perm.to(torch.int32).contiguous()
        padded = (n + 31) // 32 * 32
        fbuf = torch.zeros(3 * padded, dtype=torch.int64, device=dev)
        ebuf = torch.zeros(1, dtype=torch.float64, device=dev)
        for _ in range(3):
            kern.kernel.execute_openmm(posq, aidx, padded, box, True, True, fbuf, ebuf)
        evs = []
        for _ in range(args.steps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            kern.kernel.execute_openmm(posq, aidx, padded, box, True, True, fbuf, ebuf)
            b.record()
            evs.append((a, b))
        torch.cuda.synchronize()
        openmm_buf = {"ms_per_force_eval": round(float(np.mean([a.elapsed_time(b) for a, b in evs])), 4),
                      "note": "cf_compute_openmm on OpenMM GPU-platform buffers (double4 posq in a shuffled "
                              "atomIndex order, long long force planes of paddedNumAtoms); compare "
                              "ms_per_force_eval"}

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            log("[rank 0] timing CPU baseline sample ...")
            cpu = cpu_baseline(force, pos_np, box, args.cpu_k_sample or max(1, (k_half + 9) // 10))
        out = {
            "metric": METRIC, "value": round(ns_day, 4), "unit": "ns/day", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None,
            "dtype": "f64" if args.precision == "double" else "f32 pairs / f64 rest (mixed)", "data": "synthetic",
            "config": {"workload": f"{args.config}: periodic flexible charge-flux water box, {n} atoms, Ewald "
                                   f"rc={force.getCutoffDistance()} nm tol={force.getEwaldErrorTolerance()} "
                                   f"(alpha {alpha:.5f}, kmax {kmax[0]}, K_half {k_half}), velocity Verlet dt="
                                   f"{dt * 1000:g} fs, " + ("fp64" if args.precision == "double" else
                                                            "mixed precision (fp32 pair kernel)"),
                       "atoms": n, "kmax": list(kmax), "k_half": k_half,
                       "neighbor_skin_nm": args.neighbor_skin, "handover": args.handover, "variants": args.variants,
                       "kspace": {0: "exact k-sum, fp64 MFMA", 1: "exact k-sum, VALU",
                                  2: f"grid (ES kernel W={w_grid}, pruned DFT), same k-set"}[args.kspace_algo],
                       "nlist_builds_in_timed_steps": f"{builds1 - builds0}/{evals1 - evals0}",
                       "fp64_rescan_fallbacks_in_timed_steps": int(fb1[0] - fb0[0]),
                       "parallelism": f"atom-decomposition x{world}" + (" (RCCL all-reduce of S(k))" if world > 1 else "")},
            "ms_per_force_eval": round(ms_eval_clean, 4),
            "ms_per_harness_step": round(ms_harness, 4),
            "ms_per_force_eval_events": round(ms_eval_events, 4),
            "ms_per_force_eval_instrumented": round(ms_eval, 4),
            "graph_replay_ms_per_step": None if graph_ms is None else round(graph_ms, 4),
            "graph_stats": None if graph_ms is None else list(gstats),
            "energy_kj_mol": e_final,
            "kernels_ms_per_step": {k: round(v, 4) for k, v in per_step.items()},
            "timing_note": (f"value: K steps with HIP events around {dom} launches only; ms_per_force_eval: "
                            f"ms_per_step minus ms_per_harness_step (K steps of the MD harness alone, wall clock); "
                            f"ms_per_force_eval_events: a K-step pass with two torch events around each execute; "
                            f"kernels_ms_per_step and ms_per_force_eval_instrumented: a K-step pass with every "
                            f"phase bracketed by events and the second stream off (one stream: each phase's "
                            f"own time; kernels_roofline is from that pass)"),
            "roofline": roofline,
            "kernels_roofline": others,
            "exact_kspace": exact,
            "host_boundary": host,
            "openmm_gpu_buffers": openmm_buf,
            "cpu_baseline": cpu,
        }
        if cpu:
            out["speedup_vs_cpu_force_eval"] = round(cpu["ms_per_force_eval"] / ms_eval_clean, 1)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
