// cf_api.hip — the C-ABI (include/chargeflux.h) over the HIP kernels.
//
// cf_create  replaces ReferenceCalcCoulForceKernel::initialize (ReferenceCoulKernels.cpp:230-422)
// cf_compute replaces ReferenceCalcCoulForceKernel::execute    (ReferenceCoulKernels.cpp:424-636)
//
// Host-side work happens only in cf_create (topology, CSR gathers, Ewald parameters,
// launch plans, device allocation).  A compute call is a fixed sequence of kernel
// launches on the handle's stream with no host synchronisation (unless the caller asks
// for host outputs), so it can be captured into a hipGraph.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <exception>
#include <numeric>
#include <stdexcept>
#include <string>
#include <vector>

#include "cf_internal.h"

// Per-kernel HIP-event timing (cf_set_timing / cf_get_timing): start/stop events are
// recorded on the handle's stream around every launch, so bench.py can report kernel
// durations measured on the stream the kernels actually run on.
enum Phase { PH_FLUX, PH_PREP, PH_CELLS, PH_NLIST, PH_TABLES, PH_SFAC, PH_COEFFS, PH_FORCE, PH_DIRECT,
             PH_ASSEMBLE, PH_ENERGY, PH_GSORT, PH_GSPREAD, PH_GDFTF, PH_GDFTI, PH_GINTERP, PH_EXCL, PH_COUNT };
static const char* kPhaseNames[PH_COUNT] = {"flux_terms", "atoms_prep", "cell_sort", "neighbor_list",
                                            "kspace_tables", "kspace_sfac", "kspace_coeffs", "kspace_force",
                                            "direct_pairs", "assemble", "energy", "grid_sort", "grid_spread",
                                            "grid_dft_fwd", "grid_dft_inv", "grid_interp", "direct_excl"};
constexpr int kMaxTimed = 8192;

static void graph_forget(cf_handle* H);   // hipGraph replay cache (cf_set_graph), below
static void graph_invalidate(cf_handle* H);
struct GraphCache;
static GraphCache* graph_active(cf_handle* H);

struct cf_handle {
    cf::Handle h;
    bool timing = false;
    uint32_t timing_mask = 0xffffffffu;    // phases timed while timing is on
    std::vector<hipEvent_t> ev[PH_COUNT];  // pairs (start, stop)
    int nrec[PH_COUNT] = {};
    std::vector<void*> allocs;
    double* pos_host_dev = nullptr;   // cf_compute_host staging
    double* frc_host_dev = nullptr;
    double* ene_host_dev = nullptr;
    double* om_pos = nullptr;         // cf_compute_openmm: atom-order fp64 positions, forces, energy
    double* om_frc = nullptr;
    double* om_ene = nullptr;
    double default_box[9] = {};
    const double* pos_pending = nullptr;
    double box9_last[9] = {};   // box of the begun evaluation (graph key of its end segment)
    // host copy of the topology cf_create was given (cf_update_parameters may change only
    // parameters, not which atoms the flux terms and exclusions connect)
    std::vector<int4> topo_terms;
    std::vector<int> topo_ex_start, topo_ex_list;
    GraphCache* graph = nullptr;   // cf_set_graph (owned; freed by graph_forget)
};

namespace {

thread_local std::string g_err;

struct CfError : std::runtime_error {
    int code;
    CfError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

[[noreturn]] void fail(int code, const std::string& msg) { throw CfError(code, msg); }

template <class F>
int guarded(F&& f) {
    try {
        f();
        return CF_OK;
    } catch (const CfError& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::invalid_argument& e) {
        g_err = e.what();
        return CF_ERR_INVALID;
    } catch (const std::bad_alloc&) {
        g_err = "host allocation failed";
        return CF_ERR_NOMEM;
    } catch (const std::exception& e) {
        g_err = e.what();
        return CF_ERR_HIP;
    }
}

// Device buffers start zeroed: a list, count or index array that some evaluation reads before
// its first build holds zeros (empty rows, atom 0), never the previous owner's bytes
void zalloc(void** p, size_t bytes, const char* what) {
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) fail(CF_ERR_NOMEM, std::string(what) + ": hipMalloc failed: " + hipGetErrorString(e));
    e = hipMemset(*p, 0, bytes);
    if (e != hipSuccess) fail(CF_ERR_HIP, std::string(what) + ": hipMemset failed: " + hipGetErrorString(e));
}
template <class T>
void zalloc(T** p, size_t count, const char* what) {
    zalloc(reinterpret_cast<void**>(p), std::max<size_t>(count, 1) * sizeof(T), what);
}

// The handle's launches have drained: both of its streams (a replayed graph runs on one of them).
// Not hipDeviceSynchronize: that would also wait for the caller's other streams (torch, RCCL).
void drain_handle(const cf::Handle& h) {
    (void)hipStreamSynchronize(h.stream);
    if (h.aux) (void)hipStreamSynchronize(h.aux);
}

// Buffers are freed only once the handle's launches have drained: evaluations are asynchronous
// (the caller need not synchronize between steps) and the second stream's launches of the
// previous evaluation may still read a list that a box change reallocates
void free_idle(const cf::Handle& h, void* p) {
    if (!p) return;
    drain_handle(h);
    (void)hipFree(p);
}

template <class T>
T* dalloc(cf_handle* H, size_t count) {
    if (count == 0) count = 1;
    void* p = nullptr;
    zalloc(&p, count * sizeof(T), "device buffer");
    H->allocs.push_back(p);
    return static_cast<T*>(p);
}

template <class T>
T* dupload(cf_handle* H, const std::vector<T>& v) {
    T* p = dalloc<T>(H, v.size());
    if (!v.empty()) cf::check_hip(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice), "upload");
    return p;
}

void dfree(cf_handle* H, void* p) {
    if (!p) return;
    auto it = std::find(H->allocs.begin(), H->allocs.end(), p);
    if (it != H->allocs.end()) H->allocs.erase(it);
    free_idle(H->h, p);
}

// a buffer that captured launches point to was reallocated: the graphs are dropped now (the key's
// alloc_epoch would re-capture them anyway; dropping them here means no exec holding a freed
// address survives the reallocation)
void bump_epoch(cf_handle* H) {
    H->h.alloc_epoch++;
    graph_invalidate(H);
}

// neighbour-list capacity: the mean count within rc + skin at the density of the denser of the
// default box and the current one (v_current, 0 = not known yet), split over kSeg = 4 sub-lists,
// x2 + margin (k_excl rescans the cells for any atom that overflows, so this is a speed knob, not
// a correctness limit: a compressed box no longer sends rows to the slow rescan on every call)
void alloc_nlist(cf_handle* H, double skin, double v_current = 0.0) {
    cf::Handle& h = H->h;
    const double* b = H->default_box;
    double V = b[0] * b[4] * b[8];
    if (v_current > 0) V = std::min(V, v_current);
    double r = h.cutoff + skin;
    double mean = 4.0 / 3.0 * M_PI * r * r * r * h.n / V;
    int cap = (int)std::min<double>(h.n, 0.5 * mean + 64);
    if (h.list_capacity > 0) cap = std::max(4, std::min(cap, h.list_capacity));   // cf_options.list_capacity
    const size_t rows = std::max(h.hi - h.lo, 1);  // one row per owned atom
    // a sub-list's entries are addressed by 32-bit offsets from its row (k_nlist_wave): cap * rows
    // < 2^31 (a clamped capacity only sends more rows to the overflow rescan)
    cap = (int)std::min<size_t>((size_t)cap, ((size_t)1 << 31) / rows - 4);
    cap = (cap + 3) / 4 * 4;   // whole 4-entry chunks (list layout, cf_kernels_core.hip nl_index)
    if (h.nl && cap <= h.nb_cap) return;
    dfree(H, h.nl);
    h.nl = nullptr;
    h.nb_cap = cap;
    h.nl = dalloc<int>(H, (size_t)4 * h.nb_cap * rows);
    bump_epoch(H);
    if (!h.nl_cnt) h.nl_cnt = dalloc<int>(H, (size_t)4 * rows);
}

// getEwaldParamValue, ReferenceCoulKernels.cpp:32-35
double ewald_param_value(int kmax, double width, double alpha) {
    double t = kmax * M_PI / (width * alpha);
    return 0.05 * std::sqrt(width * alpha) * kmax * std::exp(-t * t);
}

// OpenMM's reduced box form (System::setDefaultPeriodicBoxVectors requires it): a = (ax,0,0),
// b = (bx,by,0), c = (cx,cy,cz), |bx|, |cx| <= ax/2, |cy| <= by/2.  The reference reads the
// diagonals for the reciprocal part (RCK:513-517) and the box vectors for the minimum image
// (getDeltaRPeriodic, RCK:567, 601).
void check_box_reduced(const double* b, const char* what) {
    if (b[1] != 0 || b[2] != 0 || b[5] != 0)
        fail(CF_ERR_INVALID, std::string(what) + ": box vectors must be in OpenMM's reduced form (a = (ax,0,0), b = (bx,by,0))");
    if (!(b[0] > 0 && b[4] > 0 && b[8] > 0)) fail(CF_ERR_INVALID, std::string(what) + ": box lengths must be > 0");
    if (std::fabs(b[3]) > 0.5 * b[0] || std::fabs(b[6]) > 0.5 * b[0] || std::fabs(b[7]) > 0.5 * b[4])
        fail(CF_ERR_INVALID, std::string(what) + ": box vectors must be in OpenMM's reduced form (|bx|, |cx| <= ax/2, |cy| <= by/2)");
}

// ONE_4PI_EPS0 of the OpenMM the force is evaluated for (cf_params.one_4pi_eps0; 0 = CF_ONE_4PI_EPS0)
double coulomb_constant(const cf_params* p) {
    const double ke = p->one_4pi_eps0;
    if (!(ke >= 0) || !std::isfinite(ke)) fail(CF_ERR_INVALID, "one_4pi_eps0 must be finite and >= 0 (0 = default)");
    return ke == 0 ? CF_ONE_4PI_EPS0 : ke;
}

int find_root(std::vector<int>& p, int x) {
    while (p[x] != x) { p[x] = p[p[x]]; x = p[x]; }
    return x;
}

void set_cells(cf_handle* H, const double L[3]) {
    cf::Handle& h = H->h;
    // cells per lattice direction from the box's perpendicular widths (V / |b x c|, V / |c x a|,
    // V / |a x b| for the reduced box a = (ax,0,0), b = (bx,by,0), c = (cx,cy,cz); the diagonal
    // for an orthorhombic box): a cell at least rc + skin wide in every direction puts every
    // partner of an atom in the 27 cells around its own, also for a sheared (triclinic) box,
    // whose cells are parallelepipeds in fractional coordinates (cf_kernels_core.hip k_cell_hist)
    const double bx = h.box_t[0], cx = h.box_t[1], cy = h.box_t[2];
    const double V = L[0] * L[1] * L[2];
    const double width[3] = {V / std::sqrt((L[1] * L[2]) * (L[1] * L[2]) + (bx * L[2]) * (bx * L[2]) +
                                           (bx * cy - L[1] * cx) * (bx * cy - L[1] * cx)),
                             L[1] * L[2] / std::sqrt(L[2] * L[2] + cy * cy), L[2]};
    int nc[3];
    for (int d = 0; d < 3; d++) {
        double v = std::floor((h.tric ? width[d] : L[d]) / (h.cutoff + h.list_skin));
        nc[d] = (int)std::max(1.0, std::min(v, 1024.0));
    }
    int64_t ncell = (int64_t)nc[0] * nc[1] * nc[2];
    if (ncell > h.ncell_alloc) {
        // grow (when the box grows past the initial grid).  Host side of an evaluation only, never
        // inside a capture (host_prologue runs before run_segment); graphs that point to the old
        // arrays are dropped (bump_epoch)
        bump_epoch(H);
        if (h.cell_start) { free_idle(h, h.cell_start); free_idle(h, h.cell_end); free_idle(h, h.cell_cnt); }
        if (h.own_cnt) { free_idle(h, h.own_cnt); free_idle(h, h.own_start); h.own_cnt = h.own_start = nullptr; }
        zalloc((void**)&h.cell_start, sizeof(int) * ncell, "cells");
        zalloc((void**)&h.cell_end, sizeof(int) * ncell, "cells");
        zalloc((void**)&h.cell_cnt, sizeof(int) * ncell, "cells");   // zero; re-zeroed by each build
        if (h.world > 1) {   // owned atoms per cell and their scan (list rows of a multi-rank run)
            zalloc((void**)&h.own_cnt, sizeof(int) * ncell, "cells");
            zalloc((void**)&h.own_start, sizeof(int) * (ncell + 1), "cells");
        }
        h.ncell_alloc = (int)ncell;
    }
    h.nc[0] = nc[0]; h.nc[1] = nc[1]; h.nc[2] = nc[2];
    // the per-atom lists' capacity follows the current box's density too (grows only)
    if (h.nl) alloc_nlist(H, h.list_skin, L[0] * L[1] * L[2]);
    // half neighbour list: one rank (fp64 or mixed), the wave-cooperative builder (>= 4
    // cells per axis), cells small enough for the kernel's LDS window (18 cells <= 4096 atoms,
    // with a margin for density variation: k_pairs_half flags the rare evaluation that does not
    // fit and k_excl then rescans) and sorted slots that fit the entry's 21 bits
    // cf_options.pair_list.  Several ranks with CF_PAIR_LIST_CLUSTER: the cluster-pair form, with
    // the builder keeping the cluster pairs that touch this rank's atoms (each rank evaluates those
    // once, both sides; k_excl gathers the partner-side sums of its own atoms).  Correct (the
    // multi-rank GPU tests pass with it) but slower than the full per-atom list at W = 4 / 8:
    // 0.336 / 0.304 against 0.255 / 0.197 ms rank-0 (profiles/r04ag_*): a thin slab's cells and
    // their window neighbours run whole 1024-thread blocks with the 128-KB window for few owned atoms
    const double per_cell = (double)h.n / (double)ncell;
    const bool want_cluster = h.pair_list == CF_PAIR_LIST_CLUSTER || h.pair_list == CF_PAIR_LIST_AUTO;
    h.half = h.pair_list != CF_PAIR_LIST_FULL && h.pbc &&
             (h.world == 1 || (want_cluster && h.pair_list == CF_PAIR_LIST_CLUSTER)) && nc[0] >= 4 &&
             nc[1] >= 4 && nc[2] >= 4 && per_cell * 18.0 * 1.15 <= 4096.0 && h.n < (1 << 21);
    if (h.half && ncell > h.win_cells) {
        if (h.win_out) { free_idle(h, h.win_out); free_idle(h, h.win_woff); }
        zalloc((void**)&h.win_out, sizeof(unsigned long long) * 4 * 4096 * (size_t)ncell, "half-list windows");
        zalloc((void**)&h.win_woff, sizeof(int) * 18 * (size_t)ncell, "half-list windows");
        h.win_cells = (int)ncell;
        bump_epoch(H);
    }
    // cluster-pair half list (cf_kernels_cluster.hip): one rank, fp64 and mixed,
    // wherever the per-atom half list applies.  In mixed precision its pair kernel is slower than
    // the per-atom list's (C5: 1.34 vs 1.23 ms) but its list build is 2.5x cheaper (0.07 vs 0.18 ms
    // per step): C5 2.729 against 2.815 ms/step (profiles/r05l_c5_pair_lists.txt; round 4, before the
    // skin-gated builder and the k_pairs_cq rework, the other way round: 2.878 vs 2.775).
    // CF_PAIR_LIST_ATOM_HALF keeps the per-atom list
    h.cluster = h.half && want_cluster;
    h.zcol = 0;
    if (h.cluster) {
        // within-cell z-columns of ~12 atoms (k_cell_order): clusters of 4 consecutive slots stay compact
        h.zcol = (int)std::max(1.0, std::min(8.0, std::round(std::sqrt(per_cell / 12.0))));
        const int need = h.n / 4 + (int)ncell + 1;
        // entries per i-cluster: the j-clusters whose boxes come within rc + skin in a half space
        // (cluster extent ~0.6 of the volume per cluster's edge: est = 135 at water density, rc 1,
        // skin 0.15), x2.2 + 64 for the spread (measured off the synthetic lattice: mean 166-171,
        // max 242-290, tools/cluster_proto.py); at most the clusters of one 18-cell window (k_cl_build)
        const double rho = h.n / V;
        const double ext = 0.6 * std::cbrt(4.0 / rho);
        const double rl = h.cutoff + h.list_skin + ext;
        const double est = 0.5 * 4.0 / 3.0 * M_PI * rl * rl * rl * rho / 4.0 + 8.0;
        int cap = std::min(1536, ((int)(2.2 * est) + 64 + 15) / 16 * 16);
        if (h.list_capacity > 0) cap = std::max(4, std::min(cap, h.list_capacity));   // cf_options.list_capacity
        if (need > h.ncl_cap || cap != h.cpl_cap || ncell + 1 > h.cl_cells) {
            if (h.cl_start) { free_idle(h, h.cl_start); free_idle(h, h.cl_info); free_idle(h, h.cl_bb);
                              free_idle(h, h.cpl); free_idle(h, h.cpl_cnt); }
            h.ncl_cap = std::max(need, h.ncl_cap);
            h.cpl_cap = cap;
            h.cl_cells = std::max((int)ncell + 1, h.cl_cells);
            zalloc((void**)&h.cl_start, sizeof(int) * h.cl_cells, "cluster table");
            zalloc((void**)&h.cl_info, sizeof(int2) * h.ncl_cap, "cluster table");
            zalloc((void**)&h.cl_bb, sizeof(float4) * 2 * h.ncl_cap, "cluster table");
            // (+ 64 entries: k_pairs_cq reads up to three batches of 16 past an i-cluster's count and
            // clears the ones beyond it)
            zalloc((void**)&h.cpl, sizeof(uint2) * ((size_t)h.ncl_cap * h.cpl_cap + 64), "cluster-pair list");
            zalloc((void**)&h.cpl_cnt, sizeof(int) * h.ncl_cap, "cluster-pair list");
            bump_epoch(H);
        }
        if (!h.pos4f) {
            // (+ a cluster's width, zeroed: k_pairs_cq loads all 4 slots of a listed j-cluster, a partial
            // last cluster included)
            zalloc((void**)&h.pos4f, sizeof(float4) * (h.n + 4), "fp32 positions");
            zalloc((void**)&h.slot_of, sizeof(int) * h.n, "slot map");
            bump_epoch(H);
        }
    }
}

void set_box(cf_handle* H, const double* box9) {
    cf::Handle& h = H->h;
    if (!h.pbc) { h.box_L[0] = h.box_L[1] = h.box_L[2] = 1.0; return; }
    if (!box9) fail(CF_ERR_INVALID, "periodic box required");
    check_box_reduced(box9, "current box");
    double L[3] = {box9[0], box9[4], box9[8]};
    for (int d = 0; d < 3; d++)
        if (h.cutoff > 0.5 * L[d] * (1 + 1e-12))
            fail(CF_ERR_INVALID, "cutoff exceeds half the periodic box (minimum image would be ambiguous)");
    h.box_L[0] = L[0]; h.box_L[1] = L[1]; h.box_L[2] = L[2];
    h.box_t[0] = box9[3]; h.box_t[1] = box9[6]; h.box_t[2] = box9[7];
    h.tric = box9[3] != 0 || box9[6] != 0 || box9[7] != 0;
}

// Atom decomposition: contiguous owned ranges [lo,hi), cut only where no molecule
// (connected component of flux terms + exclusions) is split, so the chain rule and the
// exclusion correction stay rank-local.
void partition(const cf_params* p, int world, int rank, int* lo, int* hi) {
    const int n = p->num_particles;
    if (world <= 1) { *lo = 0; *hi = n; return; }
    std::vector<int> par(n);
    std::iota(par.begin(), par.end(), 0);
    auto unite = [&](int a, int b) {
        if (a < 0 || a >= n || b < 0 || b >= n) fail(CF_ERR_INVALID, "particle index out of range");
        a = find_root(par, a); b = find_root(par, b);
        if (a != b) par[std::max(a, b)] = std::min(a, b);
    };
    for (int t = 0; t < p->num_flux_bonds; t++) unite(p->flux_bond_idx[2 * t], p->flux_bond_idx[2 * t + 1]);
    for (int t = 0; t < p->num_flux_angles; t++) {
        unite(p->flux_angle_idx[3 * t], p->flux_angle_idx[3 * t + 1]);
        unite(p->flux_angle_idx[3 * t], p->flux_angle_idx[3 * t + 2]);
    }
    for (int t = 0; t < p->num_flux_waters; t++) {
        unite(p->flux_water_idx[3 * t], p->flux_water_idx[3 * t + 1]);
        unite(p->flux_water_idx[3 * t], p->flux_water_idx[3 * t + 2]);
    }
    for (int k = 0; k < p->num_exceptions; k++) unite(p->exceptions[2 * k], p->exceptions[2 * k + 1]);
    std::vector<int> cmax(n, 0);
    for (int i = 0; i < n; i++) { int r = find_root(par, i); cmax[r] = std::max(cmax[r], i); }
    // cut c is valid iff every atom < c belongs to a component ending before c
    std::vector<char> valid(n + 1, 0);
    valid[0] = valid[n] = 1;
    int pm = -1;
    for (int c = 1; c < n; c++) {
        pm = std::max(pm, cmax[find_root(par, c - 1)]);
        valid[c] = pm < c;
    }
    auto nearest_cut = [&](int64_t target) {
        for (int64_t d = 0; d <= n; d++) {
            if (target - d >= 0 && valid[target - d]) return (int)(target - d);
            if (target + d <= n && valid[target + d]) return (int)(target + d);
        }
        return n;
    };
    *lo = nearest_cut((int64_t)n * rank / world);
    *hi = nearest_cut((int64_t)n * (rank + 1) / world);
    if (*hi < *lo) *hi = *lo;
}

// particles: q0 and the LJ transform (sigma/2, 2 sqrt(eps))   RCK:234-240
void parse_particles(const cf_params* p, std::vector<double>& q0, std::vector<double2>& lj) {
    const int n = p->num_particles;
    if (!p->charges || !p->sigmas || !p->epsilons) fail(CF_ERR_INVALID, "particle arrays are null");
    q0.resize(n);
    lj.resize(n);
    for (int i = 0; i < n; i++) {
        if (!(p->epsilons[i] >= 0)) fail(CF_ERR_INVALID, "epsilon must be >= 0");
        q0[i] = p->charges[i];
        lj[i] = make_double2(0.5 * p->sigmas[i], 2.0 * std::sqrt(p->epsilons[i]));
    }
}

// flux terms in reference order (bonds, angles, waters; RCK:242-284): (type, a0, a1, a2) and
// 5 parameters per term
void parse_terms(const cf_params* p, std::vector<int4>& tidx, std::vector<double>& tpar,
                 std::vector<std::vector<int>>* term_atoms) {
    const int n = p->num_particles;
    const int B = p->num_flux_bonds, A = p->num_flux_angles, W = p->num_flux_waters;
    if (B < 0 || A < 0 || W < 0) fail(CF_ERR_INVALID, "negative flux term count");
    if ((B && (!p->flux_bond_idx || !p->flux_bond_params)) || (A && (!p->flux_angle_idx || !p->flux_angle_params)) ||
        (W && (!p->flux_water_idx || !p->flux_water_params)))
        fail(CF_ERR_INVALID, "flux term arrays are null");
    auto chk = [&](int a, const char* what) {
        if (a < 0 || a >= n) fail(CF_ERR_INVALID, std::string(what) + " particle index out of range");
    };
    const int T = B + A + W;
    tidx.assign(T, make_int4(0, 0, 0, 0));
    tpar.assign((size_t)T * 5, 0.0);
    if (term_atoms) term_atoms->assign(T, {});
    for (int t = 0; t < B; t++) {
        int a0 = p->flux_bond_idx[2 * t], a1 = p->flux_bond_idx[2 * t + 1];
        chk(a0, "flux bond"); chk(a1, "flux bond");
        tidx[t] = make_int4(0, a0, a1, -1);
        tpar[5 * t] = p->flux_bond_params[2 * t]; tpar[5 * t + 1] = p->flux_bond_params[2 * t + 1];
        if (term_atoms) (*term_atoms)[t] = {a0, a1};
    }
    for (int u = 0; u < A; u++) {
        int t = B + u;
        int a0 = p->flux_angle_idx[3 * u], a1 = p->flux_angle_idx[3 * u + 1], a2 = p->flux_angle_idx[3 * u + 2];
        chk(a0, "flux angle"); chk(a1, "flux angle"); chk(a2, "flux angle");
        tidx[t] = make_int4(1, a0, a1, a2);
        tpar[5 * t] = p->flux_angle_params[2 * u]; tpar[5 * t + 1] = p->flux_angle_params[2 * u + 1];
        if (term_atoms) (*term_atoms)[t] = {a0, a1, a2};
    }
    for (int u = 0; u < W; u++) {
        int t = B + A + u;
        int a0 = p->flux_water_idx[3 * u], a1 = p->flux_water_idx[3 * u + 1], a2 = p->flux_water_idx[3 * u + 2];
        chk(a0, "flux water"); chk(a1, "flux water"); chk(a2, "flux water");
        tidx[t] = make_int4(2, a0, a1, a2);
        for (int k = 0; k < 5; k++) tpar[5 * t + k] = p->flux_water_params[5 * u + k];
        if (term_atoms) (*term_atoms)[t] = {a0, a1, a2};
    }
}

// exclusions: unique, ordered, no self pairs (std::set semantics RCK:385-391), as CSR
void parse_exclusions(const cf_params* p, std::vector<int>& exs, std::vector<int>& exl, int* max_excl) {
    const int n = p->num_particles, E = p->num_exceptions;
    if (E < 0 || (E && !p->exceptions)) fail(CF_ERR_INVALID, "bad exception list");
    std::vector<std::vector<int>> ex(n);
    for (int k = 0; k < E; k++) {
        int a0 = p->exceptions[2 * k], a1 = p->exceptions[2 * k + 1];
        if (a0 < 0 || a0 >= n || a1 < 0 || a1 >= n) fail(CF_ERR_INVALID, "exception particle index out of range");
        if (a0 == a1) continue;
        ex[a0].push_back(a1);
        ex[a1].push_back(a0);
    }
    exs.assign(n + 1, 0);
    exl.clear();
    int mx = 0;
    for (int i = 0; i < n; i++) {
        std::sort(ex[i].begin(), ex[i].end());
        ex[i].erase(std::unique(ex[i].begin(), ex[i].end()), ex[i].end());
        exs[i + 1] = exs[i] + (int)ex[i].size();
        mx = std::max(mx, (int)ex[i].size());
        exl.insert(exl.end(), ex[i].begin(), ex[i].end());
    }
    if (max_excl) *max_excl = mx;
}

// LJ types: exact-equal (sigma/2, 2 sqrt eps) pairs; <= kMaxLjTypes types ride in the
// neighbour-list entries.  Returns false when there are more.
constexpr int kMaxLjTypesHost = 64;
bool lj_types(const std::vector<double2>& lj, std::vector<int>& at, std::vector<double2>& tt) {
    const int n = (int)lj.size();
    at.assign(n, 0);
    tt.clear();
    for (int i = 0; i < n; i++) {
        int k = 0;
        while (k < (int)tt.size() && !(tt[k].x == lj[i].x && tt[k].y == lj[i].y)) k++;
        if (k == (int)tt.size()) {
            if ((int)tt.size() == kMaxLjTypesHost) return false;
            tt.push_back(lj[i]);
        }
        at[i] = k;
    }
    return true;
}

struct Timed {
    cf_handle* H; int ph; bool on;
    Timed(cf_handle* H_, int ph_)
        : H(H_), ph(ph_), on(H_->timing && ((H_->timing_mask >> ph_) & 1u) && H_->nrec[ph_] < kMaxTimed) {
        if (!on) return;
        auto& v = H->ev[ph];
        size_t need = 2 * (size_t)(H->nrec[ph] + 1);
        while (v.size() < need) {
            hipEvent_t e;
            // device-scope release: the default system-scope fence of a record writes the L2s
            // back and delays the next launch by ~10 us, which the interval then includes
            cf::check_hip(hipEventCreateWithFlags(&e, hipEventReleaseToDevice), "hipEventCreate");
            v.push_back(e);
        }
        cf::check_hip(hipEventRecord(v[2 * H->nrec[ph]], H->h.stream), "hipEventRecord");
    }
    ~Timed() {
        if (!on) return;
        (void)hipEventRecord(H->ev[ph][2 * H->nrec[ph] + 1], H->h.stream);
        H->nrec[ph]++;
    }
};

}  // namespace

namespace cf {
void check_hip(hipError_t e, const char* what) {
    if (e != hipSuccess) fail(CF_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace cf

using cf::check_hip;

extern "C" {

CF_EXPORT int cf_api_version(void) { return CF_API_VERSION; }
CF_EXPORT const char* cf_last_error(void) { return g_err.c_str(); }

CF_EXPORT int cf_create(const cf_params* p, const cf_options* opt, cf_handle** out) {
    if (out) *out = nullptr;
    cf_handle* H = nullptr;
    int rc = guarded([&] {
        if (!p || !out) fail(CF_ERR_INVALID, "null argument");
        const int n = p->num_particles;
        if (n <= 0) fail(CF_ERR_INVALID, "num_particles must be > 0");
        if (!p->charges || !p->sigmas || !p->epsilons) fail(CF_ERR_INVALID, "particle arrays are null");
        cf_options o;
        std::memset(&o, 0, sizeof(o));
        if (opt) o = *opt;
        int world = o.world_size <= 1 ? 1 : o.world_size;
        if (o.rank < 0 || o.rank >= world) fail(CF_ERR_INVALID, "rank out of range");

        int ndev = 0;
        check_hip(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
        if (ndev <= 0) fail(CF_ERR_HIP, "no HIP device available");
        if (o.device < 0 || o.device >= ndev) fail(CF_ERR_INVALID, "device ordinal out of range");
        check_hip(hipSetDevice(o.device), "hipSetDevice");

        H = new cf_handle();
        cf::Handle& h = H->h;
        h.n = n;
        h.device = o.device;
        h.rank = o.rank;
        h.world = world;
        if (o.kspace_algo < 0 || o.kspace_algo > 2) fail(CF_ERR_INVALID, "kspace_algo must be 0, 1 or 2");
        if (o.grid_width != 0 && (o.grid_width < 4 || o.grid_width > 16))
            fail(CF_ERR_INVALID, "grid_width must be 0 (default) or in [4, 16]");
        if (o.precision != CF_PRECISION_DOUBLE && o.precision != CF_PRECISION_MIXED)
            fail(CF_ERR_INVALID, "precision must be CF_PRECISION_DOUBLE or CF_PRECISION_MIXED");
        h.mixed = o.precision == CF_PRECISION_MIXED;
        if (o.handover != CF_HANDOVER_EVENT && o.handover != CF_HANDOVER_MEMORY)
            fail(CF_ERR_INVALID, "handover must be CF_HANDOVER_EVENT or CF_HANDOVER_MEMORY");
        if (o.pair_list < CF_PAIR_LIST_AUTO || o.pair_list > CF_PAIR_LIST_FULL)
            fail(CF_ERR_INVALID, "pair_list must be one of CF_PAIR_LIST_AUTO, _CLUSTER, _ATOM_HALF, _FULL "
                                 "(the octant list of API 3 was removed in API 4)");
        if (o.variants & ~(0x1F | (15 << 8))) fail(CF_ERR_INVALID, "unknown bits in variants");
        if (o.list_capacity < 0) fail(CF_ERR_INVALID, "list_capacity must be >= 0");
        // the memory hand-over is opt-in: hipStreamWaitValue64 runs as a polling kernel on this
        // runtime, so a dispatcher that serializes kernels (rocprofv3 counter collection) can run
        // the wait ahead of its producer and hold the device (a C3 --pmc pass hung, round 4); the
        // event waits are executed by the command processor and cannot starve anything
        h.handover_memory = o.handover == CF_HANDOVER_MEMORY;
        h.pair_list = o.pair_list;
        h.variants = o.variants;
        h.list_capacity = o.list_capacity;
        h.kspace_algo = o.kspace_algo;
        h.stream = (hipStream_t)o.stream;  // NULL = the null stream (orders with torch's default stream)

        // ---- particles: q0, LJ (sigma/2, 2 sqrt(eps))   RCK:234-240
        std::vector<double> q0;
        std::vector<double2> lj;
        parse_particles(p, q0, lj);

        // ---- flux terms  RCK:242-284
        const int B = p->num_flux_bonds, A = p->num_flux_angles, W = p->num_flux_waters;
        const int T = B + A + W;
        std::vector<int4> tidx;
        std::vector<double> tpar;
        std::vector<std::vector<int>> term_atoms;
        parse_terms(p, tidx, tpar, &term_atoms);
        H->topo_terms = tidx;
        h.nb = B; h.na = A; h.nw = W; h.nterms = T;
        h.nslots_dq = 2 * B + 3 * A + 3 * W;
        h.nd = 4 * B + 9 * A + 9 * W;
        // charge-delta slots -> atoms, in term order (the reference's += order RCK:61-62,113-115,191-193)
        std::vector<int> slot_atom(h.nslots_dq);
        {
            int s = 0;
            for (int t = 0; t < T; t++)
                for (int a : term_atoms[t]) slot_atom[s++] = a;
        }
        std::vector<int> qs(n + 1, 0), qslot(h.nslots_dq);
        for (int s = 0; s < h.nslots_dq; s++) qs[slot_atom[s] + 1]++;
        for (int i = 0; i < n; i++) qs[i + 1] += qs[i];
        {
            std::vector<int> fill(qs.begin(), qs.end() - 1);
            for (int s = 0; s < h.nslots_dq; s++) qslot[fill[slot_atom[s]]++] = s;
        }
        // dq/dx entries (q-atom major, x-atom minor per term, RCK:286-383) -> gather by x-atom
        std::vector<int> ent_q(h.nd), ent_x(h.nd);
        {
            int e = 0;
            for (int t = 0; t < T; t++)
                for (int u : term_atoms[t])
                    for (int v : term_atoms[t]) { ent_q[e] = u; ent_x[e] = v; e++; }
        }
        std::vector<int> cs(n + 1, 0);
        std::vector<int2> ce(h.nd);
        for (int e = 0; e < h.nd; e++) cs[ent_x[e] + 1]++;
        for (int i = 0; i < n; i++) cs[i + 1] += cs[i];
        {
            std::vector<int> fill(cs.begin(), cs.end() - 1);
            for (int e = 0; e < h.nd; e++) ce[fill[ent_x[e]]++] = make_int2(e, ent_q[e]);
        }

        // ---- exclusions: unique, ordered, no self pairs (std::set semantics RCK:385-391)
        std::vector<int> exs, exl;
        parse_exclusions(p, exs, exl, &h.max_excl);
        H->topo_ex_start = exs;
        H->topo_ex_list = exl;

        // ---- ownership for atom decomposition (see partition())
        partition(p, world, o.rank, &h.lo, &h.hi);

        // ---- Coulomb constant of the loading OpenMM (ONE_4PI_EPS0, RCK:7; 0 = the 7.x value)
        h.ke = coulomb_constant(p);

        // ---- periodic / Ewald parameters  RCK:394-421
        h.pbc = p->use_pbc ? 1 : 0;
        if (h.pbc) {
            h.cutoff = p->cutoff;
            h.tol = p->ewald_tol;
            if (!(h.cutoff > 0)) fail(CF_ERR_INVALID, "cutoff must be > 0");
            if (!(h.tol > 0 && h.tol < 0.5)) fail(CF_ERR_INVALID, "ewald tolerance must be in (0, 0.5)");
            check_box_reduced(p->default_box, "default box");
            double L[3] = {p->default_box[0], p->default_box[4], p->default_box[8]};
            for (int d = 0; d < 3; d++)
                if (h.cutoff > 0.5 * L[d] * (1 + 1e-12))
                    fail(CF_ERR_INVALID, "cutoff exceeds half the periodic box (minimum image would be ambiguous)");
            h.alpha = (1.0 / h.cutoff) * std::sqrt(-std::log(2.0 * h.tol));
            for (int d = 0; d < 3; d++) {
                int k = 1;
                while (ewald_param_value(k, L[d], h.alpha) > h.tol) k++;
                if (k % 2 == 0) k++;
                h.kmax[d] = k;
            }
            h.kg.KX = h.kmax[0];
            cf::kspace_plan(h);
            h.khalf = h.kg.k_half();
            // oversampling 2 (ng = 128 at C3, 16 tiles per axis) measured best against 1.5-3.0
            // with W adjusted for equal accuracy.  Default width: the smallest W
            // whose quadrature error (max |dF| against the exact k-sum) stays within the k-space
            // budget of a quarter of the north star's 1e-5 kJ/mol/nm, i.e. 2.5e-6, at every C3
            // configuration measured: W = 13 in fp64 (5.9e-8 at C3's initial positions; W = 12
            // reached 6.6e-6 there; W = 14: 6.9e-8 at +3-4 % step time), W = 8 in mixed precision
            // (bar: 1e-4 RMS relative)
            if (h.kspace_algo == 2) cf::grid_plan(h, o.grid_width ? o.grid_width : (h.mixed ? 8 : 13), 2.0);
        }

        // ---- device allocation + upload
        h.q0 = dupload(H, q0);
        h.lj = dupload(H, lj);
        h.term_idx = dupload(H, tidx);
        h.term_par = dupload(H, tpar);
        h.dq_slot = dalloc<double>(H, h.nslots_dq);
        h.qcsr_start = dupload(H, qs);
        h.qcsr_slot = dupload(H, qslot);
        h.dqdx = dalloc<double>(H, (size_t)3 * h.nd);
        h.ccsr_start = dupload(H, cs);
        h.ccsr_ent = dupload(H, ce);
        h.ex_start = dupload(H, exs);
        h.ex_list = dupload(H, exl);
        h.q = dalloc<double>(H, n);
        h.dedq_self = dalloc<double>(H, n);
        h.dedq = dalloc<double>(H, n);
        h.e_atom = dalloc<double>(H, (size_t)3 * n);
        h.f_part = dalloc<double>(H, (size_t)3 * n);
        h.terms_dev = dalloc<double>(H, 4);
        h.e_part = dalloc<double>(H, 3 * ((size_t)n / 256 + 2));
        h.energy_dev = dalloc<double>(H, 1);
        h.e_ticket = dalloc<int>(H, cf::kNumTickets);
        h.err_dev = dalloc<int>(H, 1);
        check_hip(hipHostMalloc((void**)&h.err_host, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent),
                  "hipHostMalloc (guard word)");
        *h.err_host = 0;
        check_hip(hipHostGetDevicePointer((void**)&h.err_host_dev, h.err_host, 0), "hipHostGetDevicePointer");
        check_hip(hipMemset(h.e_ticket, 0, sizeof(int) * cf::kNumTickets), "memset");
        check_hip(hipMemset(h.dedq, 0, sizeof(double) * n), "memset");
        check_hip(hipMemset(h.f_part, 0, sizeof(double) * 3 * n), "memset");
        check_hip(hipMemset(h.e_atom, 0, sizeof(double) * 3 * n), "memset");
        check_hip(hipMemset(h.terms_dev, 0, sizeof(double) * 4), "memset");
        int nown = h.hi - h.lo;
        if (h.pbc) {
            const cf::KGeom& g = h.kg;
            h.tric = p->default_box[3] != 0 || p->default_box[6] != 0 || p->default_box[7] != 0;
            h.box_t[0] = p->default_box[3]; h.box_t[1] = p->default_box[6]; h.box_t[2] = p->default_box[7];
            set_cells(H, std::vector<double>{p->default_box[0], p->default_box[4], p->default_box[8]}.data());
            h.erfc_tab = dupload(H, cf::erfc_table(h.alpha * h.cutoff * (1.0 + 1e-9), &h.erfc_scale, &h.erfc_m));
            if (h.mixed) {
                h.erfc_tab_f = dupload(H, cf::erfc_table_f(h.alpha * h.cutoff * (1.0 + 1e-6), &h.erfc_scale_f, &h.erfc_m_f));
            }
            h.cell_key = dalloc<int>(H, n); h.cell_key_sorted = dalloc<int>(H, n);
            h.atom_val = dalloc<int>(H, n); h.atom_sorted = dalloc<int>(H, n);
            h.pos4s = dalloc<double4>(H, n);
            h.ljs = dalloc<double2>(H, n);
            // LJ types: exact-equal (sigma/2, 2 sqrt eps) pairs; <= 64 types ride in the list entries
            {
                std::vector<int> at;
                std::vector<double2> tt;
                if (lj_types(lj, at, tt)) {
                    h.lj_ntypes = (int)tt.size();
                    h.atom_type = dupload(H, at);
                    h.lj_tab = dalloc<double2>(H, kMaxLjTypesHost);   // capacity for cf_update_parameters
                    check_hip(hipMemcpy(h.lj_tab, tt.data(), sizeof(double2) * tt.size(), hipMemcpyHostToDevice),
                              "upload LJ types");
                    h.typ_s = dalloc<int>(H, n);
                }
            }
            h.key_tmp = dalloc<int>(H, n);
            h.atom_tmp = dalloc<int>(H, n);
            h.skin_flag = dalloc<int>(H, 1);
            check_hip(hipMemset(h.skin_flag, 0, sizeof(int)), "memset");
            h.half_flag = dalloc<int>(H, 1);
            check_hip(hipMemset(h.half_flag, 0, sizeof(int)), "memset");
            h.n_builds_dev = dalloc<long long>(H, 1);
            check_hip(hipMemset(h.n_builds_dev, 0, sizeof(long long)), "memset");
            h.n_fallback_dev = dalloc<long long>(H, 3);
            check_hip(hipMemset(h.n_fallback_dev, 0, 3 * sizeof(long long)), "memset");
            if (h.world > 1) h.own_s = dalloc<int>(H, std::max(nown, 1));  // owned atoms, cell-sorted
            std::copy(p->default_box, p->default_box + 9, H->default_box);
            alloc_nlist(H, 0.0);
            if (h.kspace_algo == 0) {
                // phase tables: padded rows stay zero forever (memset once)
                h.tab_xq = dalloc<double2>(H, (size_t)h.npad * g.KX);
                h.tab_y = dalloc<double2>(H, (size_t)h.npad * g.NYP);
                h.tab_cs = dalloc<double>(H, (size_t)g.NB * h.npad * g.CSW);
                check_hip(hipMemset(h.tab_xq, 0, sizeof(double2) * h.npad * g.KX), "memset");
                check_hip(hipMemset(h.tab_y, 0, sizeof(double2) * h.npad * g.NYP), "memset");
                check_hip(hipMemset(h.tab_cs, 0, sizeof(double) * g.NB * h.npad * g.CSW), "memset");
                h.s_slab = dalloc<double>(H, (size_t)h.sp.nchunks * 2 * g.nslots() * g.NZP);
                h.s_red = dalloc<double>(H, (size_t)2 * g.nslots() * g.NZP);
                size_t ncoef = (size_t)g.nmtiles() * g.nksteps() * 64;
                h.coef_a = dalloc<double>(H, ncoef);
                check_hip(hipMemset(h.coef_a, 0, sizeof(double) * ncoef), "memset coef");
                h.t_part = dalloc<double>(H, (size_t)h.fp.nparts() * nown * 4);
                h.e_rec_part = dalloc<double>(H, (size_t)(g.KX * g.NY * g.KZ + 255) / 256 + 1);
            } else if (h.kspace_algo == 2) {
                const cf::GridPlan& gp = h.gp;
                const size_t npts = (size_t)gp.ng[0] * gp.ng[1] * gp.ng[2];
                if (npts >= (size_t)INT_MAX)   // the grid kernels index with 32-bit ints
                    fail(CF_ERR_INVALID, "k-space grid too large (more than 2^31 points)");
                std::vector<double2> tw[3], tw8[3];
                std::vector<double> dc[3];
                cf::grid_tables(h, tw, tw8, dc);
                for (int d = 0; d < 3; d++) {
                    h.g_tw[d] = dupload(H, tw[d]);
                    h.g_deconv[d] = dupload(H, dc[d]);
                    if (!tw8[d].empty()) h.g_tw8[d] = dupload(H, tw8[d]);
                }
                h.g_grid = dalloc<double>(H, npts);
                h.g_t1 = dalloc<double2>(H, (size_t)gp.ng[0] * gp.ng[1] * gp.KZ);
                h.g_t2 = dalloc<double2>(H, (size_t)gp.ng[0] * gp.NY * gp.KZ);
                h.g_b = dalloc<double2>(H, (size_t)gp.NX * gp.NY * gp.KZ);
                h.g_cnt = dalloc<int>(H, gp.nbins);
                check_hip(hipMemset(h.g_cnt, 0, sizeof(int) * gp.nbins), "memset");   // re-zeroed by k_g_scatter
                h.g_start = dalloc<int>(H, gp.nbins + 1);
                const size_t no = std::max(nown, 1);
                h.g_srec = dalloc<double4>(H, no);
                h.g_g0u = dalloc<int4>(H, no);
                h.g_rank = dalloc<int>(H, no);
                h.g_tmp = dalloc<int>(H, no);
                h.g_order = dalloc<int>(H, no);
                h.g_g0s = dalloc<int4>(H, no);
                h.g_taps = dalloc<double>(H, no * 72);
                // W <= 9: k_g_order_taps stores points 0..15 of each row only; 16..23 stay zero
                check_hip(hipMemset(h.g_taps, 0, sizeof(double) * no * 72), "memset taps");
                if (h.world > 1) {
                    // [0..2] the slab (min, max first tap, reference tap); then k_g_bin's per-block
                    // (min, max), one pair per block of its launch (<= one block per 256 owned atoms)
                    h.g_xrange = dalloc<int>(H, 3 + 2 * ((size_t)no / 256 + 1));
                    const int init[3] = {INT_MAX, INT_MIN, 0};
                    check_hip(hipMemcpy(h.g_xrange, init, sizeof(init), hipMemcpyHostToDevice), "x-slab init");
                }
                h.t_part = dalloc<double>(H, no * 4);
                // energy partials: k_g_coeffs' blocks of 256 modes, or the fused forward x stage's blocks
                // of >= 16 sequences (one rank, launch_grid_dft_fwd)
                h.e_rec_part = dalloc<double>(H, std::max<size_t>((size_t)(gp.NX * gp.NY * gp.KZ + 255) / 256,
                                                                  (size_t)gp.NY * gp.KZ / 16 + 2) + 1);
            } else {
                int blocks_k = (int)((h.khalf + 255) / 256);
                h.sk_nchunk = std::max(1, std::min((2048 + blocks_k - 1) / blocks_k, std::max(1, nown / 256)));
                h.kvec = dalloc<double4>(H, h.khalf);
                h.sk_slab = dalloc<double>(H, (size_t)h.sk_nchunk * 2 * h.khalf);
                h.sk_red = dalloc<double>(H, (size_t)2 * h.khalf);
                h.t_part = dalloc<double>(H, (size_t)nown * 4);
                h.e_rec_part = dalloc<double>(H, (size_t)(h.khalf + 255) / 256 + 1);
            }
        }
        check_hip(hipDeviceSynchronize(), "create sync");
        *out = H;
    });
    if (rc != CF_OK && H) {
        for (void* p2 : H->allocs) (void)hipFree(p2);
        if (H->h.err_host) (void)hipHostFree(H->h.err_host);
        delete H;
    }
    return rc;
}

CF_EXPORT int cf_destroy(cf_handle* H) {
    if (!H) return CF_OK;
    return guarded([&] {
        (void)hipSetDevice(H->h.device);
        drain_handle(H->h);   // both streams' launches, and any graph still running
        graph_forget(H);
        for (void* p : H->allocs) (void)hipFree(p);
        for (auto& v : H->ev)
            for (hipEvent_t e : v) (void)hipEventDestroy(e);
        if (H->h.win_out) { (void)hipFree(H->h.win_out); (void)hipFree(H->h.win_woff); }
        if (H->h.cl_start) { (void)hipFree(H->h.cl_start); (void)hipFree(H->h.cl_info); (void)hipFree(H->h.cl_bb);
                             (void)hipFree(H->h.cpl); (void)hipFree(H->h.cpl_cnt); }
        if (H->h.pos4f) { (void)hipFree(H->h.pos4f); (void)hipFree(H->h.slot_of); }
        if (H->h.cell_start) (void)hipFree(H->h.cell_start);
        if (H->h.cell_end) (void)hipFree(H->h.cell_end);
        if (H->h.cell_cnt) (void)hipFree(H->h.cell_cnt);
        if (H->h.own_cnt) { (void)hipFree(H->h.own_cnt); (void)hipFree(H->h.own_start); }
        if (H->h.own_stream) (void)hipStreamDestroy(H->h.stream);
        if (H->h.aux) (void)hipStreamDestroy(H->h.aux);
        if (H->h.ev_fork) (void)hipEventDestroy(H->h.ev_fork);
        if (H->h.ev_join) (void)hipEventDestroy(H->h.ev_join);
        if (H->h.err_host) (void)hipHostFree(H->h.err_host);
        delete H;
    });
}

CF_EXPORT int cf_partition(const cf_params* p, int32_t world_size, int32_t rank, int32_t* lo, int32_t* hi) {
    return guarded([&] {
        if (!p || !lo || !hi) fail(CF_ERR_INVALID, "null argument");
        if (p->num_particles <= 0) fail(CF_ERR_INVALID, "num_particles must be > 0");
        int world = world_size <= 1 ? 1 : world_size;
        if (rank < 0 || rank >= world) fail(CF_ERR_INVALID, "rank out of range");
        int l = 0, h = 0;
        partition(p, world, rank, &l, &h);
        *lo = l; *hi = h;
    });
}

CF_EXPORT int cf_set_neighbor_skin(cf_handle* H, double skin) {
    return guarded([&] {
        if (!H) fail(CF_ERR_INVALID, "null handle");
        if (!(skin >= 0 && skin < 1e3)) fail(CF_ERR_INVALID, "skin must be finite and >= 0");
        cf::Handle& h = H->h;
        if (h.pending_flags >= 0) fail(CF_ERR_STATE, "cf_set_neighbor_skin during a begun evaluation");
        check_hip(hipSetDevice(h.device), "hipSetDevice");
        check_hip(hipStreamSynchronize(h.stream), "stream sync");
        h.skin = skin;
        h.list_valid = false;
        bump_epoch(H);   // captured graphs baked in the old list state (pos_ref, capacity): re-capture
        if (!h.pbc) return;
        alloc_nlist(H, skin);
        if (skin > 0 && !h.pos_ref) h.pos_ref = dalloc<double>(H, (size_t)3 * h.n);
    });
}

// updateParametersInContext for CoulForce (the reference has none): new
// charges, LJ parameters and flux-term parameters on the same topology.
CF_EXPORT int cf_update_parameters(cf_handle* H, const cf_params* p) {
    return guarded([&] {
        if (!H || !p) fail(CF_ERR_INVALID, "null argument");
        cf::Handle& h = H->h;
        if (h.pending_flags >= 0) fail(CF_ERR_STATE, "cf_update_parameters during a begun evaluation");
        if (p->num_particles != h.n) fail(CF_ERR_INVALID, "the number of particles has changed");
        if ((p->use_pbc ? 1 : 0) != h.pbc) fail(CF_ERR_INVALID, "periodicity cannot be changed by an update");
        if (h.pbc && (p->cutoff != h.cutoff || p->ewald_tol != h.tol))
            fail(CF_ERR_INVALID, "the cutoff and Ewald tolerance cannot be changed by an update");
        if (coulomb_constant(p) != h.ke)
            fail(CF_ERR_INVALID, "the Coulomb constant (one_4pi_eps0) cannot be changed by an update");
        std::vector<double> q0;
        std::vector<double2> lj;
        parse_particles(p, q0, lj);
        std::vector<int4> tidx;
        std::vector<double> tpar;
        parse_terms(p, tidx, tpar, nullptr);
        bool same = tidx.size() == H->topo_terms.size();
        for (size_t t = 0; same && t < tidx.size(); t++) {
            const int4 a = tidx[t], b = H->topo_terms[t];
            same = a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w;
        }
        if (!same) fail(CF_ERR_INVALID, "the flux terms' particles have changed (only parameters can be updated)");
        std::vector<int> exs, exl;
        parse_exclusions(p, exs, exl, nullptr);
        if (exs != H->topo_ex_start || exl != H->topo_ex_list)
            fail(CF_ERR_INVALID, "the set of excluded pairs has changed (only parameters can be updated)");
        check_hip(hipSetDevice(h.device), "hipSetDevice");
        check_hip(hipStreamSynchronize(h.stream), "stream sync");
        check_hip(hipMemcpy(h.q0, q0.data(), sizeof(double) * h.n, hipMemcpyHostToDevice), "upload charges");
        check_hip(hipMemcpy(h.lj, lj.data(), sizeof(double2) * h.n, hipMemcpyHostToDevice), "upload LJ");
        if (!tpar.empty())
            check_hip(hipMemcpy(h.term_par, tpar.data(), sizeof(double) * tpar.size(), hipMemcpyHostToDevice),
                      "upload flux parameters");
        if (h.typ_s) {
            std::vector<int> at;
            std::vector<double2> tt;
            if (lj_types(lj, at, tt)) {
                h.lj_ntypes = (int)tt.size();
                check_hip(hipMemcpy(h.atom_type, at.data(), sizeof(int) * h.n, hipMemcpyHostToDevice), "upload types");
                check_hip(hipMemcpy(h.lj_tab, tt.data(), sizeof(double2) * tt.size(), hipMemcpyHostToDevice),
                          "upload LJ types");
            } else {
                h.typ_s = nullptr;   // more than 64 LJ parameter sets now: per-atom LJ gathers
                h.lj_ntypes = 0;
            }
        }
        h.list_valid = false;   // sorted LJ / types are refreshed by the next list build
        bump_epoch(H);          // lj_ntypes / typ_s are kernel arguments of captured graphs: re-capture
    });
}

CF_EXPORT int cf_get_neighbor_stats(const cf_handle* H, int64_t* builds, int64_t* evaluations) {
    if (!H) { g_err = "null handle"; return CF_ERR_INVALID; }
    if (builds) {
        long long b = 0;
        if (H->h.n_builds_dev) {
            (void)hipSetDevice(H->h.device);
            if (hipMemcpy(&b, H->h.n_builds_dev, sizeof(b), hipMemcpyDeviceToHost) != hipSuccess) {
                g_err = "hipMemcpy failed";
                return CF_ERR_HIP;
            }
        }
        *builds = b;
    }
    if (evaluations) *evaluations = H->h.n_evals;
    return CF_OK;
}

CF_EXPORT int cf_get_pair_list(const cf_handle* H, int32_t* kind) {
    if (!H || !kind) { g_err = "null argument"; return CF_ERR_INVALID; }
    const cf::Handle& h = H->h;
    *kind = !h.pbc || h.nc[0] == 0 ? CF_PAIR_LIST_AUTO
                                   : (h.cluster ? CF_PAIR_LIST_CLUSTER : (h.half ? CF_PAIR_LIST_ATOM_HALF : CF_PAIR_LIST_FULL));
    return CF_OK;
}

CF_EXPORT int cf_get_fallback_stats(const cf_handle* H, int64_t* half_list_fallbacks, int64_t* rows_rescanned,
                                    int32_t* reasons) {
    if (!H) { g_err = "null handle"; return CF_ERR_INVALID; }
    long long v[3] = {0, 0, 0};
    if (H->h.n_fallback_dev) {
        (void)hipSetDevice(H->h.device);
        if (hipStreamSynchronize(H->h.stream) != hipSuccess ||
            hipMemcpy(v, H->h.n_fallback_dev, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) {
            g_err = "hipMemcpy failed";
            return CF_ERR_HIP;
        }
    }
    if (half_list_fallbacks) *half_list_fallbacks = v[0];
    if (rows_rescanned) *rows_rescanned = v[1];
    if (reasons) *reasons = (int32_t)v[2];
    return CF_OK;
}

CF_EXPORT int cf_get_ewald_params(const cf_handle* H, double* alpha, int32_t kmax[3]) {
    if (!H) { g_err = "null handle"; return CF_ERR_INVALID; }
    if (alpha) *alpha = H->h.alpha;
    if (kmax) { kmax[0] = H->h.kmax[0]; kmax[1] = H->h.kmax[1]; kmax[2] = H->h.kmax[2]; }
    return CF_OK;
}

CF_EXPORT int cf_get_grid_shape(const cf_handle* H, int32_t ng[3], int32_t* width) {
    if (!H) { g_err = "null handle"; return CF_ERR_INVALID; }
    const bool grid = H->h.pbc && H->h.kspace_algo == 2;
    if (ng)
        for (int d = 0; d < 3; d++) ng[d] = grid ? H->h.gp.ng[d] : 0;
    if (width) *width = grid ? H->h.gp.W : 0;
    return CF_OK;
}

CF_EXPORT int cf_get_owned_range(const cf_handle* H, int32_t* lo, int32_t* hi) {
    if (!H) { g_err = "null handle"; return CF_ERR_INVALID; }
    if (lo) *lo = H->h.lo;
    if (hi) *hi = H->h.hi;
    return CF_OK;
}

// Host side of one evaluation (no launches): the box, the neighbour-list decision and the
// cell geometry (set_cells may allocate), bookkeeping.  Neighbour list: rebuilt on every call
// (skin 0, the reference's behaviour, RCK:559), or kept while no atom has moved more than half
// the skin.  The host forces a rebuild (first call, new box, skin change); otherwise
// k_atoms_prep checks the displacements on the device and the cell commit / list kernels follow
// its flag, so nothing waits on the host and the launches are graph-capturable.
static bool host_prologue(cf_handle* H, const double* box9) {
    cf::Handle& h = H->h;
    set_box(H, box9);
    if (h.pbc) std::memcpy(H->box9_last, box9, sizeof(H->box9_last));
    const double Lmin = std::min(h.box_L[0], std::min(h.box_L[1], h.box_L[2]));
    const double s_call = h.skin > 0 ? std::max(0.0, std::min(h.skin, 0.5 * Lmin - h.cutoff)) : 0.0;
    const bool reusable = h.pbc && h.skin > 0 && h.list_valid && s_call == h.list_skin &&
                          h.list_L[0] == h.box_L[0] && h.list_L[1] == h.box_L[1] && h.list_L[2] == h.box_L[2] &&
                          h.list_T[0] == h.box_t[0] && h.list_T[1] == h.box_t[1] && h.list_T[2] == h.box_t[2];
    if (h.pbc && !reusable) {
        h.list_skin = s_call;
        set_cells(H, h.box_L);
        h.list_valid = h.skin > 0;
        std::copy(h.box_L, h.box_L + 3, h.list_L);
        std::copy(h.box_t, h.box_t + 3, h.list_T);
    }
    h.n_evals++;
    return reusable;
}

// launches of cf_compute_begin: flux charges, cell sort + list, this rank's k-space partials
static void launch_begin(cf_handle* H, const double* pos_dev, int flags, bool reusable) {
    cf::Handle& h = H->h;
    const int forces = flags & CF_INCLUDE_FORCES, energy = flags & CF_INCLUDE_ENERGY;
    { Timed t(H, PH_FLUX); cf::launch_flux_terms(h, pos_dev); }
    { Timed t(H, PH_PREP); cf::launch_atoms_prep(h, pos_dev, reusable); }
    if (h.pbc) {
        {
            Timed t(H, PH_CELLS);
            if (!reusable) cf::launch_force_rebuild(h);
            cf::launch_cell_sort(h, pos_dev);
        }
        if (h.hi > h.lo) { Timed t(H, PH_NLIST); cf::launch_nlist(h, pos_dev); }
        if ((forces || energy) && h.hi > h.lo) {
            if (h.kspace_algo == 0) {
                { Timed t(H, PH_TABLES); cf::launch_kspace_tables(h, pos_dev); }
                { Timed t(H, PH_SFAC); cf::launch_kspace_sfac(h); }
            } else if (h.kspace_algo == 2) {
                { Timed t(H, PH_GSORT); cf::launch_grid_sort(h, pos_dev); }
                { Timed t(H, PH_GSPREAD); cf::launch_grid_spread(h); }
                { Timed t(H, PH_GDFTF); cf::launch_grid_dft_fwd(h); }
            } else {
                Timed t(H, PH_SFAC);
                cf::launch_kspace_direct_sfac(h, pos_dev);
            }
        } else if (forces || energy) {   // no owned atoms: a zero partial S(k) (all-reduced by the caller)
            int64_t cnt = 0;
            double* buf = cf::kspace_reduce_buffer(h, &cnt);
            cf::launch_zero(h, buf, cnt);   // (a kernel, not a memset node, when captured: cf_kernels_core.hip)
            if (h.kspace_algo == 1) cf::launch_kspace_kvec(h);   // read by the coefficient pass
        }
    }
}

// direct space + exclusion correction of a begun evaluation: independent of the
// structure factors, so a multi-rank caller can run it while S(k) is being all-reduced
static void launch_direct(cf_handle* H) {
    cf::Handle& h = H->h;
    if (h.hi <= h.lo) return;
    const int flags = h.pending_flags;
    const int forces = flags & CF_INCLUDE_FORCES, energy = flags & CF_INCLUDE_ENERGY;
    if (h.pbc) {
        { Timed t(H, PH_DIRECT); cf::launch_direct(h, H->pos_pending, forces); }
        { Timed t(H, PH_EXCL); cf::launch_direct_finish(h, H->pos_pending, forces); }
    } else {
        Timed t(H, PH_DIRECT);
        cf::launch_nopbc(h, H->pos_pending, forces, energy);
    }
}

// launches of cf_compute_end (after run_direct): k-space coefficients, reciprocal forces, chain
// rule + energy
static void launch_end(cf_handle* H, int flags, double* forces_dev, double* energy_dev) {
    cf::Handle& h = H->h;
    const int forces = flags & CF_INCLUDE_FORCES, energy = flags & CF_INCLUDE_ENERGY;
    const double* pos = H->pos_pending;
    // the reciprocal energy is added by rank 0 (launch_assemble_energy) from the all-reduced
    // buffer, so rank 0 runs the coefficient pass even when it owns no atoms (its begin
    // zeroed its partial buffer, which the caller's all-reduce then filled)
    if (h.pbc && (forces || energy) && (h.hi > h.lo || h.rank == 0)) {
        Timed t(H, PH_COEFFS);
        if (h.kspace_algo == 0) cf::launch_kspace_coeffs(h, energy);
        else if (h.kspace_algo == 2) cf::launch_grid_coeffs(h, energy, forces && h.hi > h.lo);   // (the inverse below)
        else cf::launch_kspace_direct_coeffs(h, energy);
    }
    if (h.hi > h.lo) {
        if (h.pbc) {
            if (forces && h.kspace_algo == 2) {
                { Timed t(H, PH_GDFTI); cf::launch_grid_dft_inv(h); }
                { Timed t(H, PH_GINTERP); cf::launch_grid_interp(h); }   // adds into dE/dq and forces
            } else if (forces) {
                Timed t(H, PH_FORCE);
                if (h.kspace_algo == 0) cf::launch_kspace_force(h, pos);
                else cf::launch_kspace_direct_force(h, pos);
                cf::launch_recip_add(h);
            }
        }
    }
    {   // chain rule (when forces are requested) and the energy reduction in one launch
        Timed t(H, PH_ENERGY);
        cf::launch_assemble_energy(h, (forces && forces_dev && h.hi > h.lo) ? forces_dev : nullptr, energy,
                                   energy_dev);
    }
}

// ---- hipGraph replay (cf_set_graph) ------------------------------------------------------------
// The launches of an evaluation are captured into hipGraphs on a private stream and replayed on
// the handle's stream while the calls look the same to the host: the same device buffers,
// flags, box and neighbour-list decision (a rebuild under a kept skin is decided on the device,
// inside the graph).  Anything else re-captures.  Segments: the whole single-call evaluation
// (cf_compute), and for the split-phase calls of a multi-rank step the begin, direct and end
// launches separately (the caller's all-reduce runs between them on the same stream).
// two-stream evaluations are captured one graph per stream chain (SEG_PRO: flux + charges,
// SEG_REC: the reciprocal chain, SEG_DCH: cell list + direct space; split-phase SEG_RFWD / SEG_REND:
// the reciprocal chain before / after the caller's all-reduce): the fork and join stay event
// operations between graph launches on the two streams, so a replay keeps the overlap (one graph
// holding both streams replayed as a single chain: 0.561 vs 0.526 ms eager at C3, round 3)
enum GraphSeg { SEG_FULL, SEG_BEGIN, SEG_DIRECT, SEG_END, SEG_PRO, SEG_REC, SEG_DCH, SEG_RFWD, SEG_REND, SEG_COUNT };

struct GraphKey {
    const void* pos = nullptr; void* frc = nullptr; void* ene = nullptr;
    int flags = -1; bool reusable = false;
    int64_t epoch = -1;   // Handle::alloc_epoch: a reallocated buffer invalidates the captured launches
    double box[9] = {};
    bool operator==(const GraphKey& o) const {
        return pos == o.pos && frc == o.frc && ene == o.ene && flags == o.flags && reusable == o.reusable &&
               epoch == o.epoch &&
               std::memcmp(box, o.box, sizeof(box)) == 0;
    }
};

struct GraphCache {
    bool enabled = false;
    hipStream_t cap = nullptr;
    hipGraphExec_t exec[SEG_COUNT] = {};
    GraphKey key[SEG_COUNT];
    bool rec_split[SEG_COUNT] = {};   // Handle::rec_split as the captured launches leave it (restored on replay)
    int64_t captures = 0, replays = 0;
    // a replaced graph may still run on one of the handle's streams (its launch arguments die with
    // it): drain them first -- the handle's streams only, not the device (the caller's torch or RCCL
    // streams are not ours to wait for)
    void drop(int s, const cf::Handle& h) {
        if (exec[s]) {
            drain_handle(h);
            (void)hipGraphExecDestroy(exec[s]);
        }
        exec[s] = nullptr;
    }
    void drop_all(const cf::Handle& h) {
        for (int s = 0; s < SEG_COUNT; s++) drop(s, h);
    }
};

// the handle's cache (one per handle, owned by it: no process-wide table whose entries could
// outlive or be confused with a destroyed handle)
static GraphCache* graph_of(cf_handle* H, bool create) {
    if (!H->graph && create) H->graph = new GraphCache();
    return H->graph;
}
static void graph_forget(cf_handle* H) {
    GraphCache* g = H->graph;
    if (!g) return;
    g->drop_all(H->h);
    if (g->cap) (void)hipStreamDestroy(g->cap);
    delete g;
    H->graph = nullptr;
}
// every captured segment is dropped (a buffer its launches point to was reallocated); the cache
// stays enabled and re-captures on the next call
static void graph_invalidate(cf_handle* H) {
    if (H->graph) H->graph->drop_all(H->h);
}
// graph mode for this call (timed evaluations run eagerly: replays could not record the events)
static GraphCache* graph_active(cf_handle* H) {
    GraphCache* g = graph_of(H, false);
    return (g && g->enabled && !H->timing) ? g : nullptr;
}

// run `launches` (which enqueue on h.stream) as segment `seg`: replay the cached graph when the
// key matches, else capture them afresh; g == null: eagerly
}  // extern "C"
template <class F>
static void run_segment(cf_handle* H, GraphCache* g, int seg, const GraphKey& k, F&& launches) {
    cf::Handle& h = H->h;
    if (!g) { launches(); return; }
    if (!g->exec[seg] || !(k == g->key[seg])) {
        g->drop(seg, h);
        hipStream_t user = h.stream;
        h.stream = g->cap;
        hipGraph_t graph = nullptr;
        hipError_t e = hipStreamBeginCapture(g->cap, hipStreamCaptureModeThreadLocal);
        if (e == hipSuccess) {
            try {
                launches();
            } catch (...) {
                (void)hipStreamEndCapture(g->cap, &graph);
                if (graph) (void)hipGraphDestroy(graph);
                h.stream = user;
                throw;
            }
            e = hipStreamEndCapture(g->cap, &graph);
        }
        h.stream = user;
        check_hip(e, "hipStreamBeginCapture / EndCapture");
        hipGraphExec_t ex = nullptr;
        e = hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        check_hip(e, "hipGraphInstantiate");   // (a failed instantiation leaves exec[seg] null)
        g->exec[seg] = ex;
        g->key[seg] = k;
        g->rec_split[seg] = h.rec_split;
        g->captures++;
    } else {
        h.rec_split = g->rec_split[seg];   // what the replayed launches leave in dedq / dedq_rec
        g->replays++;
    }
    check_hip(hipGraphLaunch(g->exec[seg], h.stream), "hipGraphLaunch");
}

extern "C" {
static GraphKey make_key(const cf::Handle& h, const void* pos, void* frc, void* ene, int flags, bool reusable,
                         const double* box9) {
    GraphKey k;
    k.pos = pos; k.frc = frc; k.ene = ene; k.flags = flags; k.reusable = reusable;
    k.epoch = h.alloc_epoch;
    if (h.pbc && box9) std::memcpy(k.box, box9, sizeof(k.box));
    return k;
}

// One single-rank evaluation.  With the grid k-space the reciprocal chain (bin sort, spread,
// forward DFT, coefficients, inverse DFT, interpolation) depends on nothing the cell list and
// the direct space produce -- both read the positions and k_atoms_prep's charges -- so it runs
// on the handle's second stream while they run on the first: the small, latency-bound launches
// of either chain (DFT stages, sorts, exclusions) fill the CUs the other leaves idle.  Joined
// before k_assemble_energy, which adds the reciprocal dE/dq and forces (stored apart by the
// interpolation) in the one-stream order: the same bits as launch_begin / direct / end.
static bool overlap_ok(const cf::Handle& h, int flags) {
    return h.overlap && h.aux && h.world == 1 && h.pbc && h.kspace_algo == 2 && h.hi > h.lo &&
           (flags & (CF_INCLUDE_FORCES | CF_INCLUDE_ENERGY));
}

// pieces of the two-stream evaluations (each enqueues on h.stream)
static void launch_prologue(cf_handle* H, const double* pos_dev, bool reusable) {
    cf::Handle& h = H->h;
    { Timed t(H, PH_FLUX); cf::launch_flux_terms(h, pos_dev); }
    { Timed t(H, PH_PREP); cf::launch_atoms_prep(h, pos_dev, reusable); }
}
// cell list + direct space + exclusions of an evaluation with these flags
static void launch_direct_chain(cf_handle* H, const double* pos_dev, int flags, bool reusable) {
    cf::Handle& h = H->h;
    {
        Timed t(H, PH_CELLS);
        if (!reusable) cf::launch_force_rebuild(h);
        cf::launch_cell_sort(h, pos_dev);
    }
    { Timed t(H, PH_NLIST); cf::launch_nlist(h, pos_dev); }
    h.pending_flags = flags;
    launch_direct(H);
    h.pending_flags = -1;
}
// the grid reciprocal chain up to the all-reduced buffer (fwd) and from it on (end); the
// interpolation stores into dedq_rec / f_rec (added by k_assemble_energy)
static void launch_rec_fwd(cf_handle* H, const double* pos_dev) {
    cf::Handle& h = H->h;
    { Timed t(H, PH_GSORT); cf::launch_grid_sort(h, pos_dev); }
    { Timed t(H, PH_GSPREAD); cf::launch_grid_spread(h); }
    { Timed t(H, PH_GDFTF); cf::launch_grid_dft_fwd(h); }
}
static void launch_rec_end(cf_handle* H, int flags) {
    cf::Handle& h = H->h;
    { Timed t(H, PH_COEFFS); cf::launch_grid_coeffs(h, flags & CF_INCLUDE_ENERGY, (flags & CF_INCLUDE_FORCES) != 0); }
    if (flags & CF_INCLUDE_FORCES) {
        { Timed t(H, PH_GDFTI); cf::launch_grid_dft_inv(h); }
        { Timed t(H, PH_GINTERP); cf::launch_grid_interp(h, true); }
    }
}
// run `launches` (a segment) on the second stream: eagerly, or as the segment's graph launched there
}  // extern "C"
template <class F>
static void on_aux(cf_handle* H, GraphCache* g, int seg, const GraphKey& k, F&& launches) {
    cf::Handle& h = H->h;
    const hipStream_t main = h.stream;
    h.stream = h.aux;
    try {
        run_segment(H, g, seg, k, launches);
    } catch (...) {
        h.stream = main;
        throw;
    }
    h.stream = main;
}
extern "C" {
// Fork / join between the caller's stream and the second stream.  Default (CF_HANDOVER_EVENT):
// agent-scope events, recorded after the producer's launches and waited on by the command
// processor (barrier packets), so no dispatch order can let a wait hold the device.
// CF_HANDOVER_MEMORY (opt-in): the producer's segment ends with k_signal (flag += 1, captured with
// the segment in graph mode) and the consumer's stream waits with hipStreamWaitValue64 for the
// count this evaluation reaches -- ~5 us cheaper per hand-over, but this runtime executes that wait
// as a polling kernel (cf_create).  Every wait is enqueued after its producer's launches, so a
// failed enqueue never leaves a wait for a signal nobody sends.
static void fork_aux(cf::Handle& h) {   // event form: record on the caller's stream, wait on the second
    check_hip(hipEventRecord(h.ev_fork, h.stream), "hipEventRecord (fork)");
    check_hip(hipStreamWaitEvent(h.aux, h.ev_fork, 0), "hipStreamWaitEvent (fork)");
}
static void wait_fork(cf::Handle& h) {   // memory form, consumer side (the producer: k_signal(sync_flag))
    check_hip(hipStreamWaitValue64(h.aux, h.sync_flag, ++h.sync_seq, hipStreamWaitValueGte, ~0ull),
              "hipStreamWaitValue64 (fork)");
}
static void join_post(cf::Handle& h) {   // event form only (the memory form: k_signal(sync_flag + 1) on aux)
    check_hip(hipEventRecord(h.ev_join, h.aux), "hipEventRecord (join)");
}
// After a failed evaluation in the memory form: the hand-over counts may be off by one (a signal
// enqueued whose wait was not, or the reverse never happens: a wait is enqueued only after its
// signal).  Every wait already enqueued has its signal enqueued before it, so draining both
// streams terminates; the counts are then read back.
static void resync_flags(cf::Handle& h) {
    if (!h.sync_flag || !h.handover_memory) return;
    (void)hipStreamSynchronize(h.stream);
    if (h.aux) (void)hipStreamSynchronize(h.aux);
    unsigned long long v[2] = {0, 0};
    if (hipMemcpy(v, h.sync_flag, sizeof(v), hipMemcpyDeviceToHost) == hipSuccess) {
        h.sync_seq = v[0];
        h.join_seq = v[1];
    }
}
// resyncs the hand-over counts when the scope is left by an exception
struct SyncGuard {
    cf::Handle& h;
    int n = std::uncaught_exceptions();
    ~SyncGuard() {
        if (std::uncaught_exceptions() > n) resync_flags(h);
    }
};
// a launch error reported after the launches of an entry point: the memory hand-over counts are
// resynchronised before the error is returned (a begin that queued its signal but failed later
// must not leave the next evaluation's wait satisfied by a stale count)
static void launch_check(cf::Handle& h, const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        resync_flags(h);
        fail(CF_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    }
}
static void join_wait(cf::Handle& h) {
    if (!h.handover_memory) {
        check_hip(hipStreamWaitEvent(h.stream, h.ev_join, 0), "hipStreamWaitEvent (join)");
        return;
    }
    check_hip(hipStreamWaitValue64(h.stream, h.sync_flag + 1, ++h.join_seq, hipStreamWaitValueGte, ~0ull),
              "hipStreamWaitValue64 (join)");
}

// Inside a capture on `cap`: an event-wait node on `ev` after everything captured so far, and
// every later captured launch after it.  (hipStreamWaitEvent on an event recorded outside the
// capture, even with hipEventWaitExternal, was refused at the end of the capture as unjoined
// work.)  The node waits, when the graph is launched, for the event's record enqueued last.
static void capture_event_wait(hipStream_t cap, hipEvent_t ev) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t graph = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t nd = 0;
    check_hip(hipStreamGetCaptureInfo_v2(cap, &st, &id, &graph, &deps, &nd), "hipStreamGetCaptureInfo_v2");
    if (st != hipStreamCaptureStatusActive || !graph) fail(CF_ERR_STATE, "capture_event_wait: stream is not capturing");
    std::vector<hipGraphNode_t> dep(deps, deps + nd);
    hipGraphNode_t w = nullptr;
    check_hip(hipGraphAddEventWaitNode(&w, graph, dep.empty() ? nullptr : dep.data(), dep.size(), ev),
              "hipGraphAddEventWaitNode");
    check_hip(hipStreamUpdateCaptureDependencies(cap, &w, 1, hipStreamSetCaptureDependencies),
              "hipStreamUpdateCaptureDependencies");
}

static void launch_full(cf_handle* H, const double* pos_dev, int flags, bool reusable, double* forces_dev,
                        double* energy_dev, GraphCache* g, const double* box9) {
    cf::Handle& h = H->h;
    // a launch that throws (capture or launch failure) must not leave the handle looking like a
    // begun evaluation (every later call would fail with CF_ERR_STATE) or on the second stream
    struct Restore {
        cf::Handle& h; hipStream_t s;
        ~Restore() { h.pending_flags = -1; h.stream = s; }
    } restore{h, h.stream};
    if (!overlap_ok(h, flags)) {
        auto one = [&] {
            h.rec_split = false;
            h.pending_flags = flags;
            launch_begin(H, pos_dev, flags, reusable);
            launch_direct(H);
            h.pending_flags = -1;
            launch_end(H, flags, forces_dev, energy_dev);
        };
        run_segment(H, g, SEG_FULL, make_key(h, pos_dev, forces_dev, energy_dev, flags, reusable, box9), one);
        return;
    }
    const int forces = flags & CF_INCLUDE_FORCES, energy = flags & CF_INCLUDE_ENERGY;
    const GraphKey key = make_key(h, pos_dev, nullptr, nullptr, flags, reusable, box9);
    auto rec = [&] {
        launch_rec_fwd(H, pos_dev);
        launch_rec_end(H, flags);
    };
    auto dch = [&] { launch_direct_chain(H, pos_dev, flags, reusable); };
    // The direct chain goes to the second stream and the reciprocal chain stays on the caller's.
    // Each hand-over costs the waiting queue ~5-15 us (tools/sync_probe.hip); this way the join's
    // wait sits behind the reciprocal chain, which ends last, so the direct chain's end is long
    // signalled when the caller's queue reaches it: C3 0.4607-0.4642 -> 0.4486-0.4504 ms/step
    // (profiles/r04q_*, the other way round)
    if (h.handover_memory) {   // two segments per evaluation (one graph per stream in graph mode)
        SyncGuard sync_guard{h};
        run_segment(H, g, SEG_PRO, key, [&] {
            launch_prologue(H, pos_dev, reusable);
            cf::launch_signal(h, h.sync_flag);
            rec();
        });
        wait_fork(h);
        on_aux(H, g, SEG_DCH, key, [&] {
            dch();
            cf::launch_signal(h, h.sync_flag + 1);
        });
        join_wait(h);
    } else {
        // the prologue's two kernels run eagerly even in graph mode: an event recorded right after
        // a graph launch reached the waiting queue ~8 us later than one after a kernel (C3 traces,
        // profiles/r06l_c3_timeline_graph_step.txt: fork gap 13.2 us against 5.0 eager)
        launch_prologue(H, pos_dev, reusable);
        fork_aux(h);
        on_aux(H, g, SEG_DCH, key, dch);
        join_post(h);
        if (g) {
            // graph mode: the join's wait (an external event-wait node: it waits for the record
            // enqueued just above, after the direct chain's graph) and the energy / chain-rule
            // kernel end the reciprocal chain's graph, so the caller's queue crosses no graph
            // boundary between the interpolation and k_assemble_energy (an eager wait and launch
            // after the graph left a ~15 us gap there, against ~6 us eager)
            const GraphKey key_rec = make_key(h, pos_dev, forces_dev, energy_dev, flags, reusable, box9);
            run_segment(H, g, SEG_REC, key_rec, [&] {
                rec();
                capture_event_wait(h.stream, h.ev_join);
                h.rec_split = forces != 0;
                cf::launch_assemble_energy(h, (forces && forces_dev) ? forces_dev : nullptr, energy, energy_dev);
            });
            h.rec_split = forces != 0;
            return;
        }
        run_segment(H, g, SEG_REC, key, rec);
        join_wait(h);
    }
    h.rec_split = forces != 0;
    Timed t(H, PH_ENERGY);
    cf::launch_assemble_energy(h, (forces && forces_dev) ? forces_dev : nullptr, energy, energy_dev);
}

// Multi-rank split-phase calls with the grid k-space: the direct chain (cell sort, list, pair
// kernels, exclusions) runs on the second stream from cf_compute_begin on, forked after
// k_atoms_prep, while the caller's stream runs the bin sort, spread and forward DFT, the
// caller's all-reduce of B(n) and, in cf_compute_end, the coefficients, inverse DFT and the
// interpolation (stored apart, as in launch_full); joined before k_assemble_energy.  So the
// latency-bound launches of a rank's small share (DFT stages over its slab, sorts) and the
// all-reduce overlap the direct space.  Results: the bits of the one-stream split-phase order.
// Graph mode captures one graph per stream chain, as launch_full.
static bool split_overlap_ok(cf_handle* H, int flags) {
    const cf::Handle& h = H->h;
    return h.overlap && h.aux && h.world > 1 && h.pbc && h.kspace_algo == 2 && h.hi > h.lo &&
           (flags & (CF_INCLUDE_FORCES | CF_INCLUDE_ENERGY));
}

static void launch_begin_split(cf_handle* H, const double* pos_dev, int flags, bool reusable, GraphCache* g,
                               const double* box9) {
    cf::Handle& h = H->h;
    const GraphKey key = make_key(h, pos_dev, nullptr, nullptr, flags, reusable, box9);
    if (h.handover_memory) {   // memory hand-overs (see fork_aux)
        SyncGuard sync_guard{h};
        run_segment(H, g, SEG_PRO, key, [&] {
            launch_prologue(H, pos_dev, reusable);
            cf::launch_signal(h, h.sync_flag);
            launch_rec_fwd(H, pos_dev);
        });
        wait_fork(h);
        try {
            on_aux(H, g, SEG_DCH, key, [&] {
                launch_direct_chain(H, pos_dev, flags, reusable);
                cf::launch_signal(h, h.sync_flag + 1);
            });
        } catch (...) {
            h.pending_flags = -1;
            throw;
        }
        return;
    }
    run_segment(H, g, SEG_PRO, key, [&] { launch_prologue(H, pos_dev, reusable); });
    fork_aux(h);
    try {
        on_aux(H, g, SEG_DCH, key, [&] { launch_direct_chain(H, pos_dev, flags, reusable); });
    } catch (...) {
        h.pending_flags = -1;
        throw;
    }
    join_post(h);
    run_segment(H, g, SEG_RFWD, key, [&] { launch_rec_fwd(H, pos_dev); });
}

static void launch_end_split(cf_handle* H, int flags, double* forces_dev, double* energy_dev, GraphCache* g,
                             const double* box9) {
    cf::Handle& h = H->h;
    const int forces = flags & CF_INCLUDE_FORCES, energy = flags & CF_INCLUDE_ENERGY;
    SyncGuard sync_guard{h};
    run_segment(H, g, SEG_REND, make_key(h, H->pos_pending, nullptr, nullptr, flags, false, box9),
                [&] { launch_rec_end(H, flags); });
    join_wait(h);
    h.rec_split = forces != 0;
    {
        Timed t(H, PH_ENERGY);
        cf::launch_assemble_energy(h, (forces && forces_dev) ? forces_dev : nullptr, energy, energy_dev);
    }
}

// the second stream and its fork / join events (created outside any capture)
static void ensure_aux(cf_handle* H) {
    cf::Handle& h = H->h;
    if (h.aux || !h.overlap || !h.pbc || h.kspace_algo != 2) return;
    check_hip(hipStreamCreateWithFlags(&h.aux, hipStreamNonBlocking), "hipStreamCreate (second stream)");
    // fork / join order two streams of this device only: an agent-scope release is enough (kernel
    // ends already release to the device; the default system-scope fence of an event record
    // writes the L2s back for host visibility, ~15-20 us per fork and per join on the timeline,
    // profiles/r04e_c3_timeline_eager_vs_graph.txt)
    const unsigned evf = hipEventDisableTiming | hipEventDisableSystemFence;
    check_hip(hipEventCreateWithFlags(&h.ev_fork, evf), "hipEventCreate");
    check_hip(hipEventCreateWithFlags(&h.ev_join, evf), "hipEventCreate");
    if (h.handover_memory && !h.sync_flag) {
        int can_wait = 0;
        if (hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, h.device) != hipSuccess ||
            !can_wait) {
            h.handover_memory = false;   // the runtime cannot wait on memory: events
        } else {
            // zeroed and drained before any wait is enqueued: the allocation may reuse a destroyed
            // handle's flags, whose old counts would satisfy this handle's first waits at once (the
            // second stream would start before its producer -- a C5 test saw wrong forces, round 4)
            h.sync_flag = dalloc<unsigned long long>(H, 2);
            check_hip(hipMemsetAsync(h.sync_flag, 0, 2 * sizeof(unsigned long long), h.aux), "sync flag init");
            check_hip(hipStreamSynchronize(h.aux), "sync flag init");
            h.sync_seq = 0;
            h.join_seq = 0;
        }
    }
    if (!h.dedq_rec) {
        h.dedq_rec = dalloc<double>(H, (size_t)h.n);
        h.f_rec = dalloc<double>(H, (size_t)4 * h.n);
        // atoms a rank does not own are never written: zero, so that cf_get_dedq adds nothing
        check_hip(hipMemset(h.dedq_rec, 0, sizeof(double) * h.n), "memset dedq_rec");
        check_hip(hipMemset(h.f_rec, 0, sizeof(double) * 4 * h.n), "memset f_rec");
    }
}

CF_EXPORT int cf_set_graph(cf_handle* H, int enable) {
    return guarded([&] {
        if (!H) fail(CF_ERR_INVALID, "null handle");
        if (H->h.pending_flags >= 0) fail(CF_ERR_STATE, "cf_set_graph during a begun evaluation");
        check_hip(hipSetDevice(H->h.device), "hipSetDevice");
        if (!enable) { graph_forget(H); return; }
        GraphCache* g = graph_of(H, true);
        g->enabled = true;
        if (!g->cap) check_hip(hipStreamCreateWithFlags(&g->cap, hipStreamNonBlocking), "hipStreamCreate (graph capture)");
    });
}

CF_EXPORT int cf_set_overlap(cf_handle* H, int enable) {
    return guarded([&] {
        if (!H) fail(CF_ERR_INVALID, "null handle");
        if (H->h.pending_flags >= 0) fail(CF_ERR_STATE, "cf_set_overlap during a begun evaluation");
        check_hip(hipSetDevice(H->h.device), "hipSetDevice");
        H->h.overlap = enable != 0;
        if (GraphCache* g = graph_of(H, false))   // captured launches follow the old stream layout
            g->drop_all(H->h);
        if (H->h.overlap) ensure_aux(H);
    });
}

CF_EXPORT int cf_get_graph_stats(const cf_handle* H, int64_t* captures, int64_t* replays) {
    GraphCache* g = graph_of(const_cast<cf_handle*>(H), false);
    if (captures) *captures = g ? g->captures : 0;
    if (replays) *replays = g ? g->replays : 0;
    return CF_OK;
}

// ---- device index guards ------------------------------------------------------------------------
// A kernel that meets an index outside the buffer it is about to address (cf_internal.h kGuard*)
// skips the access and sets a bit of Handle::err_dev; k_assemble_energy copies a nonzero value to
// the pinned, mapped err_host.  Every later entry point of the handle then fails with CF_ERR_STATE
// (sticky: the evaluation that tripped it is incomplete).  The check is one host read, no sync.
static std::string guard_names(int v) {
    static const char* names[] = {"cell bounds", "cluster table", "cluster-pair entry", "grid bins",
                                  "neighbour entry", "atom_index entry", "rebuild flag"};
    std::string s;
    for (int b = 0; b < 7; b++)
        if (v & (1 << b)) s += std::string(s.empty() ? "" : ", ") + names[b];
    return s;
}
static void guard_check(const cf::Handle& h) {
    const int v = h.err_host ? __atomic_load_n(h.err_host, __ATOMIC_ACQUIRE) : 0;
    if (v)
        fail(CF_ERR_STATE, "a device index guard tripped in an earlier evaluation (" + guard_names(v) +
                               "); its results are incomplete and the handle must be re-created");
}

// the guard bits of the handle's evaluations so far (synchronises the handle's streams)
CF_EXPORT int cf_get_device_errors(cf_handle* H, int32_t* bits) {
    return guarded([&] {
        if (!H || !bits) fail(CF_ERR_INVALID, "null argument");
        check_hip(hipSetDevice(H->h.device), "hipSetDevice");
        drain_handle(H->h);
        int v = 0;
        check_hip(hipMemcpy(&v, H->h.err_dev, sizeof(int), hipMemcpyDeviceToHost), "D2H guard word");
        *bits = v;
    });
}

// ---- the evaluation entry points -----------------------------------------------------------------
CF_EXPORT int cf_compute_begin(cf_handle* H, const double* pos_dev, const double* box9, int flags) {
    return guarded([&] {
        if (!H || !pos_dev) fail(CF_ERR_INVALID, "null argument");
        cf::Handle& h = H->h;
        if (h.pending_flags >= 0) fail(CF_ERR_STATE, "cf_compute_begin called twice without cf_compute_end");
        guard_check(h);
        check_hip(hipSetDevice(h.device), "hipSetDevice");
        const bool reusable = host_prologue(H, box9);
        ensure_aux(H);
        h.rec_split = false;
        H->pos_pending = pos_dev;
        h.split_overlap = split_overlap_ok(H, flags);
        if (h.split_overlap) {   // direct chain on the second stream (launch_begin_split)
            launch_begin_split(H, pos_dev, flags, reusable, graph_active(H), box9);
        } else {
            run_segment(H, graph_active(H), SEG_BEGIN, make_key(h, pos_dev, nullptr, nullptr, flags, reusable, box9),
                        [&] { launch_begin(H, pos_dev, flags, reusable); });
        }
        launch_check(h, "compute_begin");
        h.pending_flags = flags;
        h.direct_done = h.split_overlap;
    });
}

CF_EXPORT int cf_kspace_buffer(cf_handle* H, double** buf, int64_t* count) {
    return guarded([&] {
        if (!H || !buf || !count) fail(CF_ERR_INVALID, "null argument");
        if (!H->h.pbc) { *buf = nullptr; *count = 0; return; }
        *buf = cf::kspace_reduce_buffer(H->h, count);
    });
}

static void run_direct(cf_handle* H) {
    cf::Handle& h = H->h;
    if (h.direct_done) return;
    h.direct_done = true;
    run_segment(H, graph_active(H), SEG_DIRECT,
                make_key(h, H->pos_pending, nullptr, nullptr, h.pending_flags, false, h.pbc ? H->box9_last : nullptr),
                [&] { launch_direct(H); });
}

CF_EXPORT int cf_compute_direct(cf_handle* H) {
    return guarded([&] {
        if (!H) fail(CF_ERR_INVALID, "null handle");
        if (H->h.pending_flags < 0) fail(CF_ERR_STATE, "cf_compute_direct without cf_compute_begin");
        check_hip(hipSetDevice(H->h.device), "hipSetDevice");
        run_direct(H);
        launch_check(H->h, "compute_direct");
    });
}

CF_EXPORT int cf_compute_end(cf_handle* H, double* forces_dev, double* energy_dev) {
    return guarded([&] {
        if (!H) fail(CF_ERR_INVALID, "null handle");
        cf::Handle& h = H->h;
        if (h.pending_flags < 0) fail(CF_ERR_STATE, "cf_compute_end without cf_compute_begin");
        check_hip(hipSetDevice(h.device), "hipSetDevice");
        run_direct(H);
        const int flags = h.pending_flags;
        h.pending_flags = -1;
        if (h.split_overlap) {
            h.split_overlap = false;
            launch_end_split(H, flags, forces_dev, energy_dev, graph_active(H), h.pbc ? H->box9_last : nullptr);
        } else {
            run_segment(H, graph_active(H), SEG_END,
                        make_key(h, H->pos_pending, forces_dev, energy_dev, flags, false, h.pbc ? H->box9_last : nullptr),
                        [&] { launch_end(H, flags, forces_dev, energy_dev); });
        }
        launch_check(h, "compute_end");
    });
}

// one evaluation = begin + end; in graph mode a single-rank call is one graph (SEG_FULL)
CF_EXPORT int cf_compute(cf_handle* H, const double* pos_dev, const double* box9, int flags, double* forces_dev,
                         double* energy_dev) {
    if (H && H->h.world > 1) {
        int rc = cf_compute_begin(H, pos_dev, box9, flags);
        if (rc != CF_OK) return rc;
        return cf_compute_end(H, forces_dev, energy_dev);
    }
    return guarded([&] {
        if (!H || !pos_dev) fail(CF_ERR_INVALID, "null argument");
        cf::Handle& h = H->h;
        if (h.pending_flags >= 0) fail(CF_ERR_STATE, "cf_compute during a begun evaluation");
        guard_check(h);
        check_hip(hipSetDevice(h.device), "hipSetDevice");
        const bool reusable = host_prologue(H, box9);
        ensure_aux(H);
        H->pos_pending = pos_dev;
        launch_full(H, pos_dev, flags, reusable, forces_dev, energy_dev, graph_active(H), box9);
        h.pending_flags = -1;
        launch_check(h, "compute");
    });
}

// OpenMM GPU-platform buffers (include/chargeflux.h; the reference's CUDA platform,
// CudaCoulKernels.cpp:523-600): gather posq by atomIndex into atom-order fp64 positions, the
// device-resident evaluation, scatter the forces into the fixed-point planes and add the energy
CF_EXPORT int cf_compute_openmm(cf_handle* H, const void* posq, const void* posq_correction, int32_t posq_kind,
                                const int32_t* atom_index, int32_t padded_n, const double* box9, int flags,
                                long long* force_buf, void* energy_buf, int32_t energy_kind) {
    return guarded([&] {
        if (!H || !posq || !atom_index) fail(CF_ERR_INVALID, "null argument");
        cf::Handle& h = H->h;
        if (h.world > 1) fail(CF_ERR_STATE, "cf_compute_openmm is single-rank only");
        if (posq_kind != CF_POSQ_DOUBLE4 && posq_kind != CF_POSQ_FLOAT4)
            fail(CF_ERR_INVALID, "posq_kind must be CF_POSQ_DOUBLE4 or CF_POSQ_FLOAT4");
        if (posq_correction && posq_kind != CF_POSQ_FLOAT4)
            fail(CF_ERR_INVALID, "posq_correction goes with CF_POSQ_FLOAT4 (the mixed-precision platform)");
        if (energy_kind != CF_ENERGY_DOUBLE && energy_kind != CF_ENERGY_FLOAT)
            fail(CF_ERR_INVALID, "energy_kind must be CF_ENERGY_DOUBLE or CF_ENERGY_FLOAT");
        if (padded_n < h.n) fail(CF_ERR_INVALID, "padded_n must be >= the number of particles");
        if (h.pending_flags >= 0) fail(CF_ERR_STATE, "cf_compute_openmm during a begun evaluation");
        guard_check(h);
        check_hip(hipSetDevice(h.device), "hipSetDevice");
        if (!H->om_pos) {
            H->om_pos = dalloc<double>(H, (size_t)3 * h.n);
            H->om_frc = dalloc<double>(H, (size_t)3 * h.n);
            H->om_ene = dalloc<double>(H, 1);
        }
        const bool fw = force_buf && (flags & CF_INCLUDE_FORCES);
        cf::launch_om_gather(h, posq, posq_correction, posq_kind, atom_index, H->om_pos);
        if (fw) check_hip(hipMemsetAsync(H->om_frc, 0, sizeof(double) * 3 * h.n, h.stream), "memset forces");
        const int rc = cf_compute(H, H->om_pos, box9, flags, fw ? H->om_frc : nullptr, energy_buf ? H->om_ene : nullptr);
        if (rc != CF_OK) throw CfError(rc, g_err);
        if (fw || energy_buf)
            cf::launch_om_scatter(h, atom_index, H->om_frc, padded_n, fw ? force_buf : nullptr, H->om_ene, energy_buf,
                                  energy_kind);
        launch_check(h, "compute_openmm");
    });
}

CF_EXPORT int cf_compute_host(cf_handle* H, const double* pos_host, const double* box9, int flags,
                              double* forces_host, double* energy_host) {
    return guarded([&] {
        if (!H || !pos_host) fail(CF_ERR_INVALID, "null argument");
        if (H->h.world > 1) fail(CF_ERR_STATE, "cf_compute_host is single-rank only; use the split-phase API");
        cf::Handle& h = H->h;
        check_hip(hipSetDevice(h.device), "hipSetDevice");
        const int n = h.n;
        if (!H->pos_host_dev) {
            H->pos_host_dev = dalloc<double>(H, (size_t)3 * n);
            H->frc_host_dev = dalloc<double>(H, (size_t)3 * n);
            H->ene_host_dev = dalloc<double>(H, 1);
        }
        check_hip(hipMemcpyAsync(H->pos_host_dev, pos_host, sizeof(double) * 3 * n, hipMemcpyHostToDevice, h.stream),
                  "H2D positions");
        check_hip(hipMemsetAsync(H->frc_host_dev, 0, sizeof(double) * 3 * n, h.stream), "memset forces");
        int rc = cf_compute(H, H->pos_host_dev, box9, flags, H->frc_host_dev, H->ene_host_dev);
        if (rc != CF_OK) throw CfError(rc, g_err);
        std::vector<double> f(forces_host ? 3 * (size_t)n : 0);
        double e = 0;
        if (forces_host)
            check_hip(hipMemcpyAsync(f.data(), H->frc_host_dev, sizeof(double) * 3 * n, hipMemcpyDeviceToHost, h.stream),
                      "D2H forces");
        check_hip(hipMemcpyAsync(&e, H->ene_host_dev, sizeof(double), hipMemcpyDeviceToHost, h.stream), "D2H energy");
        check_hip(hipStreamSynchronize(h.stream), "sync");
        guard_check(h);   // (this evaluation's guards: k_assemble_energy has run)
        if (forces_host && (flags & CF_INCLUDE_FORCES))
            for (size_t k = 0; k < 3 * (size_t)n; k++) forces_host[k] += f[k];
        if (energy_host) *energy_host = e;
    });
}

CF_EXPORT int cf_get_charges(cf_handle* H, double* out) {
    return guarded([&] {
        if (!H || !out) fail(CF_ERR_INVALID, "null argument");
        check_hip(hipStreamSynchronize(H->h.stream), "sync");
        guard_check(H->h);
        check_hip(hipMemcpy(out, H->h.q, sizeof(double) * H->h.n, hipMemcpyDeviceToHost), "D2H charges");
    });
}

CF_EXPORT int cf_get_dedq(cf_handle* H, double* out) {
    return guarded([&] {
        if (!H || !out) fail(CF_ERR_INVALID, "null argument");
        check_hip(hipStreamSynchronize(H->h.stream), "sync");
        guard_check(H->h);
        check_hip(hipMemcpy(out, H->h.dedq, sizeof(double) * H->h.n, hipMemcpyDeviceToHost), "D2H dedq");
        if (H->h.rec_split) {   // (direct + excl) + rec, as k_assemble_energy adds them
            std::vector<double> r(H->h.n);
            check_hip(hipMemcpy(r.data(), H->h.dedq_rec, sizeof(double) * H->h.n, hipMemcpyDeviceToHost), "D2H dedq");
            for (int i = 0; i < H->h.n; i++) out[i] += r[i];
        }
    });
}

CF_EXPORT int cf_get_energy_terms(cf_handle* H, double terms[4]) {
    return guarded([&] {
        if (!H || !terms) fail(CF_ERR_INVALID, "null argument");
        check_hip(hipStreamSynchronize(H->h.stream), "sync");
        guard_check(H->h);
        check_hip(hipMemcpy(terms, H->h.terms_dev, sizeof(double) * 4, hipMemcpyDeviceToHost), "D2H terms");
    });
}

CF_EXPORT int cf_set_timing(cf_handle* H, int enable) {
    return guarded([&] {
        if (!H) fail(CF_ERR_INVALID, "null handle");
        check_hip(hipStreamSynchronize(H->h.stream), "sync");
        H->timing = enable != 0;
        H->timing_mask = 0xffffffffu;
        for (int p = 0; p < PH_COUNT; p++) H->nrec[p] = 0;
    });
}

CF_EXPORT int cf_set_timing_mask(cf_handle* H, uint32_t phase_mask) {
    return guarded([&] {
        if (!H) fail(CF_ERR_INVALID, "null handle");
        check_hip(hipStreamSynchronize(H->h.stream), "sync");
        H->timing = phase_mask != 0;
        H->timing_mask = phase_mask;
        for (int p = 0; p < PH_COUNT; p++) H->nrec[p] = 0;
    });
}

CF_EXPORT int cf_get_timing(cf_handle* H, int32_t max_phases, char* names, double* total_ms, int32_t* calls,
                            int32_t* nphases) {
    return guarded([&] {
        if (!H || !nphases) fail(CF_ERR_INVALID, "null argument");
        check_hip(hipStreamSynchronize(H->h.stream), "sync");
        *nphases = PH_COUNT;
        for (int p = 0; p < PH_COUNT && p < max_phases; p++) {
            double tot = 0;
            for (int k = 0; k < H->nrec[p]; k++) {
                float ms = 0;
                check_hip(hipEventElapsedTime(&ms, H->ev[p][2 * k], H->ev[p][2 * k + 1]), "hipEventElapsedTime");
                tot += ms;
            }
            if (names) { std::strncpy(names + 16 * p, kPhaseNames[p], 15); names[16 * p + 15] = 0; }
            if (total_ms) total_ms[p] = tot;
            if (calls) calls[p] = H->nrec[p];
        }
    });
}

CF_EXPORT int cf_synchronize(cf_handle* H) {
    return guarded([&] {
        if (!H) fail(CF_ERR_INVALID, "null handle");
        check_hip(hipStreamSynchronize(H->h.stream), "sync");
        guard_check(H->h);
    });
}

}  // extern "C"
