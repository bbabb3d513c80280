// cf_internal.h — device-side layout and kernel launch declarations of the MI355X
// ChargeFlux evaluator.  See DESIGN.md for the data layout in HBM and the roofline of
// each kernel.  Everything here is fp64.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/chargeflux.h"

namespace cf {

// (the Coulomb constant is a run-time value, Handle::ke: cf_params.one_4pi_eps0)
constexpr double kPi = 3.14159265358979323846;

// ---------------------------------------------------------------------------------
// k-space geometry (separable MFMA formulation)
//   combos  (nx, ny): nx in [0,KX), ny_idx in [0,NYP) with ny = ny_idx-(KY-1), valid < NY
//   columns j = 2*nz + {0:cos,1:sin}, nz in [0,KZ), padded to NZP (multiple of 16)
// ---------------------------------------------------------------------------------
struct KGeom {
    int KX = 0, KY = 0, KZ = 0;
    int NY = 0;    // 2KY-1
    int NYB = 0;   // ceil(NY/16)  (S-pass combo groups per nx)
    int NYP = 0;   // 16*NYB
    int NYB4 = 0;  // ceil(NY/4)
    int NMT = 0;   // force-pass m-tiles: ceil(KX*NY/4), combos flattened (no per-row padding)
    int NZP = 0;   // 2KZ rounded up to 16
    int NB = 0;    // column blocks of <= 64 (CS table blocks, S-pass n-blocks, force K-chunks)
    int CSW = 0;   // CS table block width: min(64, NZP)
    __host__ __device__ int nslots() const { return KX * NYP; }
    __host__ __device__ int ngroups() const { return KX * NYB; }
    __host__ __device__ int nmtiles() const { return NMT; }
    __host__ __device__ int nksteps() const { return NZP / 4; }
    __host__ __device__ int64_t k_half() const {
        return (int64_t)(KZ - 1) + (int64_t)(KY - 1) * (2 * KZ - 1) +
               (int64_t)(KX - 1) * (2 * KY - 1) * (2 * KZ - 1);
    }
};

// S-pass launch plan: workgroups = nxgroups(16 groups each) x nblocks(<=64 cols) x nchunks
struct SPassPlan {
    int wg_groups = 0;    // number of 16-group workgroup tiles
    int nchunks = 0;      // atom chunks (split-K)
    int chunk_atoms = 0;  // atoms per chunk (multiple of tile_atoms)
    int tile_atoms = 0;   // atoms staged in LDS per step (16 or 32)
    size_t lds_bytes = 0;
};

// force-pass launch plan: workgroups = atom groups x kchunks x msplit
struct FPassPlan {
    int na = 0;           // 16-atom tiles per wave
    int waves = 0;        // waves per workgroup
    int natom_groups = 0; // workgroups along atoms
    int kchunks = 0;      // K (column) chunks of <= 64
    int msplit = 0;       // m-tile range split
    int nparts() const { return kchunks * msplit; }
};

// grid path (kspace_algo = 2, cf_kernels_grid.hip): ES-kernel spreading on an oversampled
// grid of ng points per axis (multiple of 8; 8^3-point tiles = sort bins), pruned DFT to
// the reference's mode box |n_a| < K_a, interpolation
struct GridPlan {
    int W = 0;               // kernel width (grid points)
    double beta = 0;         // ES shape parameter
    double sigma = 0;        // effective oversampling min_a ng_a / (2K_a - 1)
    int ng[3] = {0, 0, 0};
    int nb[3] = {0, 0, 0};   // tiles per axis (ng/8)
    int nbins = 0;
    int KX = 0, KY = 0, KZ = 0;
    int NX = 0, NY = 0;      // 2KX-1, 2KY-1 (mode rows nx, ny in (-K, K)); nz in [0, KZ)
    // pruned DFT stages by the 8 x Q factorization (ng = 8Q; k_g_dft8_*), per axis: modes
    // per residue class k = r (mod 8) padded to mt (0: the axis uses the GEMM stages), j of the
    // first mode of class r and the class size
    int mt[3] = {0, 0, 0};
    int rj[3][8] = {}, rc[3][8] = {};
    bool dft8 = false;       // every axis qualifies and not CF_VARIANT_GEMM_DFT
    bool spread_mfma = true; // W > 9: the spread on the fp64 matrix cores, 16x8x8 tiles (CF_VARIANT_VECTOR_SPREAD: k_g_spread_tile)
    bool spread_mfma_all = false;   // CF_VARIANT_MFMA_SPREAD: the matrix form at every width
    bool interp2 = true;     // two atoms per wave, taps by DPP row broadcast (CF_VARIANT_INTERP1: k_g_interp)
    bool interp4 = true;     // W <= 8: four atoms per wave (CF_VARIANT_INTERP2: k_g_interp2)
    bool taps_f32 = false;   // mixed precision, W <= 9, vector spread: tap rows stored as fp32 (16 points)
    bool grid_f32 = false;   // mixed precision, W <= 8: the real grid stored as fp32 (spread -> z stages -> interp4)
};

struct Handle {
    // ---- configuration -------------------------------------------------------
    int n = 0;
    int pbc = 0;
    double cutoff = 1.0, tol = 1e-4, alpha = 0.0;
    double ke = CF_ONE_4PI_EPS0;   // ONE_4PI_EPS0 of the loading OpenMM (cf_params.one_4pi_eps0)
    int kmax[3] = {0, 0, 0};
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int rank = 0, world = 1;
    int lo = 0, hi = 0;  // owned atoms [lo,hi)
    int kspace_algo = 0;
    bool mixed = false;         // CF_PRECISION_MIXED: fp32 direct-space pair kernel
    KGeom kg;
    SPassPlan sp;
    FPassPlan fp;

    // ---- topology (device) ---------------------------------------------------
    double* q0 = nullptr;       // [N]
    double2* lj = nullptr;      // [N] (sigma/2, 2 sqrt(eps))
    int nb = 0, na = 0, nw = 0; // flux terms
    int nterms = 0, nslots_dq = 0, nd = 0;
    int4* term_idx = nullptr;   // [T] (type, a0, a1, a2)
    double* term_par = nullptr; // [T*5]
    double* dq_slot = nullptr;  // [S] per-term charge deltas
    int* qcsr_start = nullptr;  // [N+1] slots contributing to atom charge
    int* qcsr_slot = nullptr;
    double* dqdx = nullptr;     // [D*3] reference entry order
    int* ccsr_start = nullptr;  // [N+1] chain-rule entries by x-atom
    int2* ccsr_ent = nullptr;   // (entry, q-atom)
    int* ex_start = nullptr;    // [N+1] unique exclusion partners
    int* ex_list = nullptr;
    int max_excl = 0;

    // ---- per-evaluation work buffers -------------------------------------------
    double* q = nullptr;        // [N] realcharges
    double* dedq_self = nullptr;// [N]
    double* dedq = nullptr;     // [N] total dE/dq
    double* e_atom = nullptr;   // [N*3] per-atom (self, direct, exclusion) energy
    double* f_part = nullptr;   // [N*3] non-chain forces (recip + direct + excl)
    // single rank, grid k-space: the reciprocal chain runs on a second stream beside the cell
    // list and direct space (cf_set_overlap(h, 0): one stream); its interpolation then stores into
    // dedq_rec / f_rec, added by k_assemble_energy in the one-stream order ((direct + excl) + rec)
    bool overlap = true;
    bool rec_split = false;     // the last evaluation left the reciprocal dE/dq in dedq_rec
    bool split_overlap = false; // a begun multi-rank evaluation runs its direct chain on aux (cf_api.hip)
    hipStream_t aux = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // fork / join: agent-scope events (default), or with CF_HANDOVER_MEMORY by stream memory
    // operations (k_signal / hipStreamWaitValue64 on sync_flag[0] / [1], value = the evaluation's
    // sequence number): ~5.5 us per hand-over against ~8.5 (agent-fence event), tools/sync_probe.hip
    unsigned long long* sync_flag = nullptr;
    unsigned long long sync_seq = 0, join_seq = 0;   // the values sync_flag[0] / [1] reach this evaluation
    bool handover_memory = false;   // cf_options.handover == CF_HANDOVER_MEMORY
    double* dedq_rec = nullptr; // [N]
    double* f_rec = nullptr;    // [N][4]: the interpolated gradient p and -q (force = -q (ng/L) p)
    // cell list
    int ncell_alloc = 0;
    int nc[3] = {0, 0, 0};
    int* cell_key = nullptr; int* cell_key_sorted = nullptr;
    int* atom_val = nullptr; int* atom_sorted = nullptr;
    int* cell_start = nullptr; int* cell_end = nullptr; int* cell_cnt = nullptr;
    double4* pos4s = nullptr;   // [N] sorted wrapped (x,y,z,q)
    double2* ljs = nullptr;     // [N] sorted LJ
    int lj_ntypes = 0;          // distinct (sigma/2, 2 sqrt eps) pairs if <= 64, else 0
    int* atom_type = nullptr;   // [N] LJ type per atom
    int* typ_s = nullptr;       // [N] LJ type per sorted slot (null without types)
    double2* lj_tab = nullptr;  // [lj_ntypes]
    // persistent list with skin: pairs within rc + list_skin at the last
    // build; reused while every atom has moved <= list_skin/2 and the box is unchanged
    double skin = 0.0;          // requested skin (nm); 0 = rebuild on every evaluation
    double list_skin = 0.0;     // skin the current list was built with
    double list_L[3] = {0, 0, 0};
    double list_T[3] = {0, 0, 0};
    bool list_valid = false;
    double* pos_ref = nullptr;  // [N*3] positions at the last build (skin > 0)
    int* skin_flag = nullptr;   // [1] device: rebuild this evaluation (host-forced or moved > skin/2)
    long long* n_builds_dev = nullptr;  // [1] list builds (device counter)
    long long* n_fallback_dev = nullptr;  // [3] evaluations whose half-list sums were unusable (fp64
                                          // rescan of every atom); list rows rescanned after an
                                          // overflow; union of the half-list reasons (CF_FALLBACK_*)
    int64_t n_evals = 0;
    // device index guards (kGuard* bits): a kernel that meets an index outside the buffer it is
    // about to address sets a bit here and skips the access; k_assemble_energy copies a nonzero
    // value into err_host (pinned, mapped), which every entry point checks (cf_api.hip guard_check)
    int* err_dev = nullptr;     // [1] device
    int* err_host = nullptr;    // [1] host-mapped pinned copy (read by the host)
    int* err_host_dev = nullptr;// its device address (written by k_assemble_energy)
    // cell-sort scratch (the sort kernels run only when the device flag asks for a rebuild;
    // k_cell_commit then copies the new order to the live arrays)
    int* key_tmp = nullptr; int* atom_tmp = nullptr;
    // multi-rank: owned atoms compacted in cell-sorted order (list rows)
    int* own_s = nullptr;       // [N_own] (null on one rank: identity)
    int* own_cnt = nullptr;     // [ncell] owned atoms per cell (multi-rank; re-zeroed by k_cell_scatter)
    int* own_start = nullptr;   // [ncell + 1] their exclusive scan: first list row of each cell
    int nb_cap = 0;             // capacity of each of the 4 neighbour sub-lists of an atom
    int* nl = nullptr;          // [4][nb_cap][N] transposed sub-lists (sorted index | shift<<26)
    int* nl_cnt = nullptr;      // [4][N]
    // half list: one rank, fp64, >= 4 cells per axis
    bool half = false;
    int64_t alloc_epoch = 0;    // bumped when a buffer a captured graph may point to is reallocated
    int* half_flag = nullptr;   // [1] device: half-list sums unusable this evaluation (fp64 rescan)
    unsigned long long* win_out = nullptr;   // [ncell][4096][4] window partials (fixed point)
    int* win_woff = nullptr;    // [ncell][18]
    int win_cells = 0;          // cells win_out / win_woff are sized for
    // cluster-pair half list (cf_kernels_cluster.hip): one rank, same window and
    // fixed-point j side as the half list; clusters = runs of <= 4 consecutive sorted slots of one cell
    bool cluster = false;
    int pair_list = CF_PAIR_LIST_AUTO;   // cf_options.pair_list
    int list_capacity = 0;      // cf_options.list_capacity (0: automatic)
    int variants = 0;           // cf_options.variants (CF_VARIANT_*)
    int block_rounds() const { return (variants >> 8) & 15; }   // k_g_bin / k_assemble_energy rounds (0: by N)
    int zcol = 0;               // columns per cell axis of the within-cell sort (k_cell_order; 0 = atom order)
    int ncl_cap = 0;            // cluster capacity: N/4 + ncell
    int cl_cells = 0;           // cells cl_start is sized for (+1)
    int* cl_start = nullptr;    // [ncell + 1] first cluster of each cell
    int2* cl_info = nullptr;    // [ncl_cap] (first sorted slot, atom count)
    float4* cl_bb = nullptr;    // [ncl_cap][2] bounding box (lo, hi) at the last list build
    int cpl_cap = 0;            // cluster-pair entries per i-cluster
    uint2* cpl = nullptr;       // [ncl_cap][cpl_cap] (first slot of j | window cell << 21, pair mask)
    int* cpl_cnt = nullptr;     // [ncl_cap]
    float4* pos4f = nullptr;    // [N] sorted wrapped fp32 (x, y, z, LJ type bits)
    int* slot_of = nullptr;     // [N] atom -> sorted slot (exclusion masks of the list build)
    // k-space (MFMA path)
    int npad = 0;               // owned rows of the phase tables, padded to the S-pass tile
    double2* tab_xq = nullptr;  // [Nown][KX]
    double2* tab_y = nullptr;   // [Nown][NYP]
    double* tab_cs = nullptr;   // [Nown][NZP]
    double* s_slab = nullptr;   // [nchunks][2][slots][NZP]
    double* s_red = nullptr;    // [2][slots][NZP]  <- all-reduced buffer
    double* coef_a = nullptr;   // [mtiles][ksteps][64]
    double* t_part = nullptr;   // [nparts][Nown][4]
    double* e_rec_part = nullptr; // [nblk]
    int e_rec_nblk = 0;
    int coef_inv = 0;           // several ranks: the next inverse x stage applies the coefficients (1; 2: and
                                // writes the energy partials) -- set by launch_grid_coeffs
    // k-space (grid path)
    GridPlan gp;
    double* g_grid = nullptr;   // [ngx][ngy][ngz] spread charges, later the potential grid
    double2* g_t1 = nullptr;    // [ngx][ngy][KZ]
    double2* g_t2 = nullptr;    // [ngx][NY][KZ]
    double2* g_b = nullptr;     // [NX][NY][KZ] B(n) (all-reduced), then coefficients f(n)
    double2* g_tw[3] = {nullptr, nullptr, nullptr};  // [2K-1][ng] e^{i 2pi n g/ng}
    double2* g_tw8[3] = {nullptr, nullptr, nullptr};  // [8 r][Q b][mt] e^{i 2pi b k/ng}, k the class-r modes
    double* g_deconv[3] = {nullptr, nullptr, nullptr};  // [K] 1/phih(n/ng)
    int* g_cnt = nullptr;       // [nbins]
    int* g_start = nullptr;     // [nbins+1]
    double4* g_srec = nullptr;  // [Nown] (s_x, s_y, s_z, q), s = grid coordinate
    int4* g_g0u = nullptr;      // [Nown] first tap (unwrapped) per axis, bin
    int* g_rank = nullptr;      // [Nown]
    int* g_tmp = nullptr;       // [Nown]
    int* g_order = nullptr;     // [Nown] sorted slot -> owned index
    int4* g_g0s = nullptr;      // [Nown] wrapped first taps per sorted slot
    double* g_taps = nullptr;   // [Nown][72]
    int* g_xrange = nullptr;    // [3] multi-rank x-slab of the owned atoms' taps (null on one rank)
    // k-space (direct VALU check path)
    int64_t khalf = 0;
    double* sk_slab = nullptr;  // [nchunk][2][khalf]
    double* sk_red = nullptr;   // [2][khalf]
    double4* kvec = nullptr;    // [khalf] (kx,ky,kz, w=2*c*eak)
    int sk_nchunk = 0;
    // energy
    double* erfc_tab = nullptr;  // erfcx interval polynomials (cf_kernels_core.hip erfc_table)
    double erfc_scale = 0; int erfc_m = 0;
    double erfc_scale_f = 0; int erfc_m_f = 0;   // fp32 table (mixed precision): its own interval width
    float* erfc_tab_f = nullptr; // fp32 erfcx table (mixed precision)
    double* terms_dev = nullptr; // [4]
    double* e_part = nullptr;    // [ceil(Nown/256)][3] energy block partials
    double* energy_dev = nullptr;// [1] internal
    int* e_ticket = nullptr;     // [kNumTickets] last-block tickets (0 between launches)
    // state
    int pending_flags = -1;     // flags of a begun evaluation
    bool direct_done = false;   // cf_compute_direct already ran for the begun evaluation
    double box_L[3] = {0, 0, 0};
    double box_t[3] = {0, 0, 0};   // reduced triclinic box off-diagonals (bx, cx, cy); 0 = orthorhombic
    bool tric = false;             // any off-diagonal nonzero: cells in fractional coordinates, box-vector minimum image
};

// ---- launchers (cf_kernels_*.hip) ------------------------------------------------
std::vector<double> erfc_table(double xmax, double* scale, int* m);     // width 1/16, degree 7, fp64 pair kernel
std::vector<float> erfc_table_f(double xmax, double* scale, int* m);    // degree 6, mixed-precision kernel
std::vector<double> erfc_table_deg(double xmax, int deg, double width, int max_m, double* scale, int* m);
void launch_flux_terms(Handle& h, const double* pos);
void launch_atoms_prep(Handle& h, const double* pos, bool skin_check);   // q, self term [, skin_flag |= moved > list_skin/2]
void launch_cell_sort(Handle& h, const double* pos);
void launch_force_rebuild(Handle& h);                   // skin_flag = 1 (a kernel: graph-capture safe)
void launch_zero(Handle& h, double* p, int64_t n);      // p[0, n) = 0 (a kernel: graph-capture safe)
void launch_nlist(Handle& h, const double* pos);
void launch_cluster_list(Handle& h);                   // cluster table, bounding boxes, cluster-pair list (rebuild only)
void launch_pairs_cluster(Handle& h, const double* pos, int include_forces);   // k_pairs_cq
void launch_cluster_table(Handle& h);                  // k_cl_scan + k_cl_bbox (rebuild only)
void launch_direct(Handle& h, const double* pos, int include_forces);          // the pair kernel
void launch_direct_finish(Handle& h, const double* pos, int include_forces);   // overflow rescan + exclusions
void launch_recip_add(Handle& h);   // dedq, f_part += reciprocal partials
void launch_nopbc(Handle& h, const double* pos, int include_forces, int include_energy);
void launch_signal(Handle& h, unsigned long long* flag);   // one-thread kernel: *flag += 1 (system-scope release)
void launch_assemble_energy(Handle& h, double* forces_out, int include_energy, double* energy_out);   // chain rule (forces_out != null) + energy

void kspace_plan(Handle& h);
size_t kspace_alloc_bytes(const Handle& h);
void launch_kspace_tables(Handle& h, const double* pos);
void launch_kspace_sfac(Handle& h);
double* kspace_reduce_buffer(Handle& h, int64_t* count);
void launch_kspace_coeffs(Handle& h, int include_energy);
void launch_kspace_force(Handle& h, const double* pos);

// direct VALU reference path of the reciprocal sum (kspace_algo = 1)
void launch_kspace_kvec(Handle& h);   // k-vectors and weights of the current box (direct path)
void launch_kspace_direct_sfac(Handle& h, const double* pos);
void launch_kspace_direct_coeffs(Handle& h, int include_energy);
void launch_kspace_direct_force(Handle& h, const double* pos);

// grid path (kspace_algo = 2)
void grid_plan(Handle& h, int width, double sigma);
void grid_tables(const Handle& h, std::vector<double2> tw[3], std::vector<double2> tw8[3], std::vector<double> deconv[3]);
void launch_grid_sort(Handle& h, const double* pos);
void launch_grid_spread(Handle& h);
void launch_grid_dft_fwd(Handle& h);
double* grid_reduce_buffer(Handle& h, int64_t* count);
void launch_grid_coeffs(Handle& h, int include_energy, bool inverse_follows);
void launch_grid_dft_inv(Handle& h);
void launch_grid_interp(Handle& h, bool split = false);   // split: store into dedq_rec / f_rec

// OpenMM GPU-platform buffers (cf_kernels_openmm.hip, cf_compute_openmm)
void launch_om_gather(Handle& h, const void* posq, const void* corr, int posq_kind, const int* atom_index,
                      double* pos);
void launch_om_scatter(Handle& h, const int* atom_index, const double* frc, int padded, long long* fbuf,
                       const double* ene, void* ebuf, int energy_kind);

void check_hip(hipError_t e, const char* what);

// ---- fp64 math helpers shared by the pair and grid kernels -------------------------
// 1/sqrt(r2): hardware v_rsq_f64 estimate (relative error 5.3e-8 on MI355X, tools/rsq_probe.hip)
// + one Newton step -> 4.3e-15 relative (a second step would give 2.4e-16; the pair terms'
// other roundings and the 1e-5 kJ/mol/nm force bar make it unnecessary)
// Kernels whose 8-B LDS reads load the LDS pipe keep them as single ds_read_b64 (2 LDS cycles
// per wave-instruction on gfx950) instead of letting the compiler pair them into ds_read2_b64
// (8 cycles for the pair: half the bandwidth; MI355X_MICROARCH.md, LDS table)
// (a gfx950 code-generation feature: the host pass, which only sees the launch stub, has no such
// feature and gets nothing)
#if defined(__HIP_DEVICE_COMPILE__)
#define CF_LDS_UNPAIRED __attribute__((target("no-load-store-opt")))
#else
#define CF_LDS_UNPAIRED
#endif

__device__ __forceinline__ double rsqrt_fp64(double r2) {
    double y = __builtin_amdgcn_rsq(r2);
    return y * fma(-0.5 * r2 * y, y, 1.5);
}

// d = a*b + c as one VOP3 v_fma_f64.  For a Horner step with a constant addend the compiler
// otherwise emits v_mov_b64 (constant -> accumulator) + v_fmac_f64: one extra VALU op per step.
// c is a wave-uniform constant: an SGPR pair operand (round 5; held in VGPRs, the twelve exp
// coefficients took 24 VGPRs of the 128 the pair kernels may use: 32-40 B/lane of spills, none now)
__device__ __forceinline__ double fma3(double a, double b, double c) {
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
    return d;
}

// e^y for y in [-700, 0] (no overflow / NaN handling needed there): y = k ln2 + r with
// |r| <= ln2/2 (Cody-Waite split of ln2), e^r by its degree-12 Taylor polynomial (truncation
// < 2e-16 relative), times 2^k.  17 VALU instructions against ~35 for the libm exp, whose
// range checks and coefficient register copies this path does not need (fma3 keeps the
// Horner steps with VGPR-held constants as single VOP3 FMAs).
__device__ __forceinline__ double exp_nonpos(double y) {
    const double k = rint(y * 1.4426950408889634);
    double r = fma(-k, 6.93147180369123816490e-01, y);
    r = fma(-k, 1.90821492927058770002e-10, r);
    double p = 2.0876756987868098979e-09;
    p = fma3(p, r, 2.5052108385441718775e-08);
    p = fma3(p, r, 2.7557319223985890653e-07);
    p = fma3(p, r, 2.7557319223985888276e-06);
    p = fma3(p, r, 2.4801587301587301566e-05);
    p = fma3(p, r, 1.9841269841269841253e-04);
    p = fma3(p, r, 1.3888888888888888889e-03);
    p = fma3(p, r, 8.3333333333333332177e-03);
    p = fma3(p, r, 4.1666666666666664354e-02);
    p = fma3(p, r, 1.6666666666666665741e-01);
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    return ldexp(p, (int)k);
}

// Workgroups are dispatched round-robin over the 8 XCDs (block b -> XCD b % 8), each XCD with
// its own L2.  This maps the blocks one XCD receives onto a contiguous 1/8 of the logical
// block range, so cell-sorted atoms (spatially coherent) share that XCD's L2 with their
// neighbours.  A bijection on [0, gridDim.x) for any grid size.
constexpr int kNumXcd = 8;
__device__ __forceinline__ int xcd_block() {
    const int b = blockIdx.x, nb = gridDim.x;
    const int x = b % kNumXcd, per = nb / kNumXcd, rem = nb % kNumXcd;
    return x * per + min(x, rem) + b / kNumXcd;
}

// last-block tickets (Handle::e_ticket[]): the energy reduction, the cell-count bounds, the
// grid-bin bounds
constexpr int kTicketEnergy = 0, kTicketCells = 1, kTicketGrid = 2, kNumTickets = 4;

// device index guards (Handle::err_dev): each bit names the invariant that failed; the kernel
// skips the access it guards.  All of these hold by construction -- a set bit is a bug (or
// corrupted device memory), reported as CF_ERR_STATE by the next entry point (cf_api.hip)
constexpr int kGuardCellBounds = 1;    // k_cell_order: a cell's member range past the atom count
constexpr int kGuardClusterTable = 2;  // k_cl_scan: more clusters than the cluster table holds
constexpr int kGuardListEntry = 4;     // k_cl_build / k_pairs_cq: a list entry's slot or window cell out of range
constexpr int kGuardGridBins = 8;      // k_g_bin / k_g_order_taps: bin bounds past the owned atom count
constexpr int kGuardNeighbor = 16;     // k_nlist / k_nlist_wave: a partner slot past the atom count
constexpr int kGuardAtomIndex = 32;    // k_om_gather: an OpenMM atomIndex entry outside [0, N) (caller data)
constexpr int kGuardRebuildFlag = 64;  // k_cell_commit: the rebuild flag clear on a handle without a skin

// ---- counting-sort helpers shared by the cell and grid-bin sorts ----------------------
// atomicAdd(&cnt[key], 1) aggregated over runs of equal keys in consecutive lanes (spatially
// ordered atoms put long runs of a wave in one cell or bin, whose counter would otherwise
// serialize up to 64 atomics): the first lane of each run adds the run length, all runs'
// atomics in flight at once (one round trip), and the run's lanes take consecutive ranks.
// Any set of lanes may be valid (a run starts after an invalid lane).  Returns a provisional
// rank within the key; the sorts fix the final order in a separate, deterministic pass.
__device__ __forceinline__ int wave_agg_inc(int* cnt, int key, bool valid) {
    const int lane = threadIdx.x & 63;
    const int prev = __shfl_up(valid ? key : -1, 1);   // -1: no key (keys are >= 0)
    const bool head = valid && (lane == 0 || prev != key);
    const unsigned long long cut = __ballot(head || !valid);        // run starts + invalid lanes
    const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);   // bits 0..lane
    const int leader = 63 - __clzll((long long)(cut & upto));        // start of this lane's run
    const unsigned long long after = cut & ~upto;
    const int next = after ? __ffsll((long long)after) - 1 : 64;     // first lane past this run
    int base = 0;
    if (head) base = atomicAdd(&cnt[key], next - lane);
    base = __shfl(base, leader);
    return base + (lane - leader);
}

// Last-block-done: true (in every thread) for the block that finishes last; it re-arms the
// ticket.  Every thread of the block must call it.  The data the last block reads from the
// other blocks must be device-scope atomics (RMWs whose results the threads waited for, or
// agent-scope atomic stores followed by a wait), read back with agent-scope atomic loads
// (ld_agent): then no release/acquire fence is needed, whose L2 writeback in every block
// cost more than the kernels themselves (measured: 375-block grid sort 10 -> 39 us).
__device__ __forceinline__ bool last_block_done(int* ticket) {
    __shared__ bool last;
    __builtin_amdgcn_s_waitcnt(0);   // this wave's atomic stores are performed
    __syncthreads();
    if (threadIdx.x == 0) {
        last = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1;
        if (last) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return last;
}

template <class T>
__device__ __forceinline__ T ld_agent(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void st_agent(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// exclusive scan of one int per thread over a block of NT threads (NT a multiple of 64, at
// most 1024; sh: NT ints of LDS, left holding the block total in sh[NT - 1]): wave scans by
// shuffles, then the wave totals -- 4 barriers (a Hillis-Steele scan over LDS takes 2 log2 NT)
template <int NT>
__device__ __forceinline__ int block_exclusive_scan_t(int v, int* sh) {
    constexpr int NW = NT / 64;
    static_assert(NT % 64 == 0 && NW <= 16, "block scan: NT must be a multiple of 64, at most 1024");
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    __syncthreads();   // a previous scan's readers of sh are done
    if (lane == 63) sh[w] = x;
    __syncthreads();
    int before = 0, total = 0;
#pragma unroll
    for (int k = 0; k < NW; k++) {
        const int s = sh[k];
        before += k < w ? s : 0;
        total += s;
    }
    __syncthreads();
    if (t == NT - 1) sh[NT - 1] = total;
    __syncthreads();
    return before + x - v;
}

// counts cnt[0..m) (device-scope atomics of other blocks: read with ld_agent) -> start[c]
// (and end[c] = start[c + 1] when end != null; start[m] = total when total_at_end), by the NT
// threads of one block, in tiles of 8 NT counts: each thread issues the loads of kBoundsU
// tiles at once (one memory latency per kBoundsU tiles, not one per count or per tile: the
// C5 grid's 32k bins are 16 tiles at NT = 256).  Returns the total (in every thread).
constexpr int kBoundsU = 4;
template <int NT>
__device__ __forceinline__ int block_counts_to_bounds(int m, int* cnt, int* start, int* end, bool total_at_end,
                                                       int* sh) {
    __shared__ int tile[8 * NT];
    const int t = threadIdx.x;
    int carry = 0;
    for (int sbase = 0; sbase < m; sbase += kBoundsU * 8 * NT) {
        int vu[kBoundsU][8];
#pragma unroll
        for (int u = 0; u < kBoundsU; u++)
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int c = sbase + u * 8 * NT + k * NT + t;
                vu[u][k] = c < m ? ld_agent(cnt + c) : 0;
            }
#pragma unroll
        for (int u = 0; u < kBoundsU; u++) {
            const int base = sbase + u * 8 * NT;
            if (base >= m) break;   // block-uniform
#pragma unroll
            for (int k = 0; k < 8; k++) tile[k * NT + t] = vu[u][k];
            __syncthreads();
            int v[8];
            int sum = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) { v[k] = tile[8 * t + k]; sum += v[k]; }
            int run = carry + block_exclusive_scan_t<NT>(sum, sh);
            carry += sh[NT - 1];   // inclusive total of the tile
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int c = base + 8 * t + k;
                if (c < m) {
                    start[c] = run;
                    run += v[k];
                    if (end) end[c] = run;
                }
            }
            __syncthreads();
        }
    }
    if (total_at_end && t == 0) start[m] = carry;
    return carry;
}

}  // namespace cf
