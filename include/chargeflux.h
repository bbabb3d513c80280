/*
 * chargeflux.h — C-ABI boundary of the MI355X-native ChargeFlux (CoulForce) evaluator.
 *
 * This is the drop-in boundary for the reference's hot path
 *   CoulPlugin::CalcCoulForceKernel::{initialize, execute}
 *   (reference: openmmapi/include/CoulKernels.h:15-38,
 *    platforms/reference/src/ReferenceCoulKernels.cpp:230-636).
 *
 * Plain C: pointers, sizes and int error codes only.  No C++ exceptions, no torch
 * types cross it.  An OpenMM plugin or a ctypes/cffi binding
 * calls these functions; the Python mirror `openmmcoul` in this repo does exactly that.
 *
 * Units follow the reference (OpenMM): nm, e, kJ/mol, rad.  All arithmetic is fp64.
 */
#ifndef CHARGEFLUX_H_
#define CHARGEFLUX_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(_WIN32)
#define CF_EXPORT __declspec(dllexport)
#else
#define CF_EXPORT __attribute__((visibility("default")))
#endif

#define CF_API_VERSION 4   /* 2: cf_params.one_4pi_eps0; 3: cf_options.handover, pair_list, variants, list_capacity;
                              4: device index guards (cf_get_device_errors), cf_compute_openmm, octant list removed */

/* Error codes (negative).  cf_last_error() returns the message of the last failure
 * on the calling thread.  Mirrors the reference's OpenMMException paths. */
#define CF_OK 0
#define CF_ERR_INVALID -1  /* bad argument / parameter validation failed     */
#define CF_ERR_HIP -2      /* a HIP runtime call failed                       */
#define CF_ERR_STATE -3    /* call sequence error (e.g. end without begin)    */
#define CF_ERR_NOMEM -4    /* device allocation failed                        */

/* Coulomb constant ONE_4PI_EPS0 (kJ mol^-1 nm e^-2).  The reference takes it from the
 * OpenMM it is compiled against (openmm/reference/SimTKOpenMMRealType.h, included at
 * ReferenceCoulKernels.cpp:7; used at :508, :517, :580-589, :608-619), so its value depends on
 * the OpenMM version: 138.935456 in OpenMM 7.x headers, 138.93545764438198 (CODATA 2018) in
 * OpenMM 8.x.  cf_params.one_4pi_eps0 carries the loading OpenMM's value; 0 selects the
 * default below (OpenMM 7.x). */
#define CF_ONE_4PI_EPS0 138.935456
#define CF_ONE_4PI_EPS0_CODATA2018 138.93545764438198

/*
 * Force parameters: the flat storage of CoulPlugin::CoulForce
 * (reference: openmmapi/include/CoulForce.h:138-149, openmmapi/src/CoulForce.cpp:12-140).
 * Arrays are host memory, read only during cf_create.
 */
typedef struct cf_params {
    int32_t num_particles;
    const double* charges;  /* [N]  addParticle(charge, ...)          CoulForce.cpp:18-22 */
    const double* sigmas;   /* [N]  LJ sigma (nm)                                          */
    const double* epsilons; /* [N]  LJ epsilon (kJ/mol)                                    */

    int32_t num_exceptions;
    const int32_t* exceptions; /* [2E] excluded pairs (p1,p2)         CoulForce.cpp:56-68 */

    int32_t num_flux_bonds;
    const int32_t* flux_bond_idx;    /* [2B] (p1,p2)                  CoulForce.cpp:78-94   */
    const double* flux_bond_params;  /* [2B] (k [e/nm], b [nm])                             */
    int32_t num_flux_angles;
    const int32_t* flux_angle_idx;   /* [3A] (p1,p2,p3), p2 central   CoulForce.cpp:96-114  */
    const double* flux_angle_params; /* [2A] (k [e/rad], theta0 [rad])                      */
    int32_t num_flux_waters;
    const int32_t* flux_water_idx;   /* [3W] (O,H1,H2)                CoulForce.cpp:116-140 */
    const double* flux_water_params; /* [5W] (k1,k2,kub [e/nm], b0,ub0 [nm])                */

    int32_t use_pbc;          /* setUsesPeriodicBoundaryConditions   CoulForce.cpp:52-54   */
    double cutoff;            /* setCutoffDistance (nm), PBC only                          */
    double ewald_tol;         /* setEwaldErrorTolerance                                    */
    double default_box[9];    /* System::getDefaultPeriodicBoxVectors, rows a,b,c (nm);
                                 kmax is derived from THIS box (ReferenceCoulKernels.cpp:399-420) */
    double one_4pi_eps0;      /* Coulomb constant of the OpenMM the force is evaluated for
                                 (its ONE_4PI_EPS0); 0 = CF_ONE_4PI_EPS0.  Must be >= 0, finite */
} cf_params;

/* Execution options (all-zero = single GPU, device 0, default stream). */
typedef struct cf_options {
    int32_t device;      /* HIP device ordinal                                             */
    void* stream;        /* hipStream_t to enqueue on (NULL = the null stream)             */
    int32_t rank;        /* atom-decomposition rank (0..world_size-1)                       */
    int32_t world_size;  /* 0 or 1 = single GPU                                            */
    int32_t kspace_algo; /* reciprocal sum of ReferenceCoulKernels.cpp:513-556:
                            0 = default: exact k-sum, fp64 MFMA separable form
                            1 = exact k-sum, direct VALU sincos (check path)
                            2 = grid: the same k-sum through ES-kernel spreading, pruned DFT
                                and interpolation (error set by grid_width) */
    int32_t grid_width;  /* kspace_algo 2: ES kernel width in grid points, 4..16 (0 = 13, or 8 mixed) */
    int32_t precision;   /* CF_PRECISION_DOUBLE (0, default) or CF_PRECISION_MIXED (1): the
                            direct-space pair kernel computes in fp32 (positions, erfc, LJ) and
                            accumulates forces in fp32 and energies in fp64 per atom; every
                            other term stays fp64.  Accuracy target: RMS
                            relative force error <= 1e-4 against the fp64 build. */
    int32_t handover;    /* fork / join of the handle's second stream (grid k-space, see cf_set_overlap):
                            CF_HANDOVER_EVENT (0, default): hipEvents, waited on by the command
                            processor -- safe under any dispatch order;
                            CF_HANDOVER_MEMORY (1): a one-thread counter kernel + hipStreamWaitValue64,
                            ~5 us per hand-over cheaper, but the runtime executes the wait as a
                            polling kernel, so a tool that serializes dispatches (rocprofv3 counter
                            collection) can deadlock it.  Same results either way. */
    int32_t pair_list;   /* direct-space neighbour list (periodic):
                            CF_PAIR_LIST_AUTO (0): cluster-pair half list on one rank (fp64 and mixed),
                              per-atom full list on several ranks;
                            CF_PAIR_LIST_CLUSTER (1): the cluster-pair half list wherever its cell window
                              fits (also mixed precision, and several ranks with an ownership filter);
                            CF_PAIR_LIST_ATOM_HALF (2): the per-atom half list on one rank (full on several);
                            CF_PAIR_LIST_FULL (3): the per-atom full (two-sided) list.
                            (API 3's CF_PAIR_LIST_OCTANT (4) was removed in API 4: CF_ERR_INVALID.)
                            Same pair set and the same results up to the fp64 summation order. */
    int32_t variants;    /* CF_VARIANT_* bits: alternative kernels of the same sums, kept for A/B
                            verification (0 = the production kernels) */
    int32_t list_capacity;   /* neighbour-list capacity cap: cluster-pair entries per i-cluster, and
                            entries per sub-list of the per-atom lists; 0 = automatic (the density of
                            the denser of the default and the current box).  A list that overflows it
                            is evaluated by the fp64 rescan (slow, same results; tests force it). */
    int32_t reserved[1];
} cf_options;

#define CF_PRECISION_DOUBLE 0
#define CF_PRECISION_MIXED 1

#define CF_HANDOVER_EVENT 0
#define CF_HANDOVER_MEMORY 1

#define CF_PAIR_LIST_AUTO 0
#define CF_PAIR_LIST_CLUSTER 1
#define CF_PAIR_LIST_ATOM_HALF 2
#define CF_PAIR_LIST_FULL 3

/* cf_options.variants (grid k-space; each equal to the production kernel to <= 1e-12 relative) */
#define CF_VARIANT_GEMM_DFT 1        /* the DFT stages as fp64-MFMA complex GEMMs (k_g_cgemm), not the
                                        8 x Q factorized stages (also used when a grid exceeds those) */
#define CF_VARIANT_VECTOR_SPREAD 2   /* W > 9: the VALU spread (k_g_spread_tile), not the matrix cores */
#define CF_VARIANT_MFMA_SPREAD 4     /* W <= 9: the matrix-core spread (k_g_spread_mfma) */
#define CF_VARIANT_INTERP1 8         /* one atom per wave interpolation (k_g_interp) */
#define CF_VARIANT_INTERP2 16        /* W <= 8: two atoms per wave (k_g_interp2), not four */
#define CF_VARIANT_BLOCK_ROUNDS(r) (((r) & 15) << 8)   /* grid bin sort and energy kernels: r rounds of
                                        256 atoms per block (1..8; 0 = by N) */

/* compute flags */
#define CF_INCLUDE_FORCES 1
#define CF_INCLUDE_ENERGY 2

typedef struct cf_handle cf_handle;

CF_EXPORT int cf_api_version(void);
CF_EXPORT const char* cf_last_error(void);

/* Replaces ReferenceCalcCoulForceKernel::initialize (ReferenceCoulKernels.cpp:230-422). */
CF_EXPORT int cf_create(const cf_params* params, const cf_options* options, cf_handle** out);
CF_EXPORT int cf_destroy(cf_handle* h);

/* Ewald parameters chosen at initialize: alpha (nm^-1) and odd kmax per axis
 * (ReferenceCoulKernels.cpp:32-35, 401-420). */
CF_EXPORT int cf_get_ewald_params(const cf_handle* h, double* alpha, int32_t kmax[3]);
/* Grid of the kspace_algo 2 reciprocal path: points per axis and the ES kernel width
 * (zeros for the exact k-sum paths and without PBC). */
CF_EXPORT int cf_get_grid_shape(const cf_handle* h, int32_t ng[3], int32_t* width);
/* Owned atom range [lo, hi) of this rank (all atoms when world_size <= 1). */
CF_EXPORT int cf_get_owned_range(const cf_handle* h, int32_t* lo, int32_t* hi);
/* Host-only (no device needed): the atom decomposition cf_create would use.  Ranges are
 * contiguous and never split a molecule (connected component of flux terms + exceptions). */
CF_EXPORT int cf_partition(const cf_params* params, int32_t world_size, int32_t rank, int32_t* lo, int32_t* hi);

/* Persistent neighbour list (the reference rebuilds its voxel-hash list on
 * every call, ReferenceCoulKernels.cpp:559).  skin = 0 (default): rebuild on every
 * evaluation.  skin > 0 (nm): the list holds pairs within cutoff + skin and is kept while
 * the box is unchanged and no atom has moved more than skin/2 since the last build (decided
 * on the device).  The evaluated pair set is identical either way (every pair is tested
 * against the exact cutoff); only the fp64 summation order can differ.  Positions must be
 * continuous between calls (a re-wrapped atom just triggers a rebuild).  The skin is capped
 * at half the smallest box length minus the cutoff. */
CF_EXPORT int cf_set_neighbor_skin(cf_handle* h, double skin);
/* updateParametersInContext (the reference's CoulForce has none): replace
 * the charges, LJ parameters and flux-term parameters of a created handle.  The topology
 * must be unchanged -- the same particle count, flux terms on the same particles in the same
 * order, the same set of excluded pairs -- and so must periodicity, cutoff and Ewald
 * tolerance (alpha and kmax stay those of cf_create); otherwise CF_ERR_INVALID.  The next
 * evaluation rebuilds the neighbour list.  Not allowed between cf_compute_begin and _end. */
CF_EXPORT int cf_update_parameters(cf_handle* h, const cf_params* params);
/* The direct-space list the handle evaluates with (cf_options.pair_list resolved for this system and
 * box: CF_PAIR_LIST_CLUSTER, CF_PAIR_LIST_ATOM_HALF or CF_PAIR_LIST_FULL; CF_PAIR_LIST_AUTO before the
 * first periodic evaluation and without periodic boundaries).  A cluster or per-atom half list that
 * does not fit the box (fewer than 4 cells per axis, an 18-cell window over 4096 atoms at the
 * density of the box, several ranks without CF_PAIR_LIST_CLUSTER) resolves to CF_PAIR_LIST_FULL. */
CF_EXPORT int cf_get_pair_list(const cf_handle* h, int32_t* kind);
/* Number of neighbour-list builds and evaluations since cf_create. */
CF_EXPORT int cf_get_neighbor_stats(const cf_handle* h, int64_t* builds, int64_t* evaluations);
/* Slow-path diagnostics since cf_create (synchronises the stream): evaluations whose half-list
 * partner sums could not be used, so that every atom's pair sums were recomputed by the fp64 cell
 * rescan (same results, several times slower); list rows rescanned after a full-list overflow;
 * and the union of the reasons for the first (CF_FALLBACK_* bits).  Nonzero values on a
 * production system mean the neighbour-list capacity or the cell geometry does not suit it
 * (DESIGN.md §4.4).  Any output may be NULL. */
#define CF_FALLBACK_WINDOW 1        /* a cell's 18-cell window held more than 4096 atoms */
#define CF_FALLBACK_LIST 2          /* a list row overflowed, or the builder could not place it */
#define CF_FALLBACK_FIXED_POINT 4   /* a partner-side term beyond the fixed-point range (|F| >= 2^16) */
CF_EXPORT int cf_get_fallback_stats(const cf_handle* h, int64_t* half_list_fallbacks, int64_t* rows_rescanned,
                                    int32_t* reasons);

/* Device index guards.  The kernels check the data-dependent indices they are about to address
 * (cell and grid-bin bounds, the cluster table, list entries) against the buffers they index;
 * an index outside its buffer -- impossible by construction, so a bug or corrupted device
 * memory -- skips the access and sets a CF_GUARD_* bit instead of faulting the GPU.  The bit is
 * copied to host-mapped memory at the end of the evaluation, and every later entry point of the
 * handle (cf_compute*, cf_synchronize, cf_get_charges / _dedq / _energy_terms; cf_compute_host in
 * the same call) then returns CF_ERR_STATE naming the guard.  Sticky: re-create the handle.
 * cf_get_device_errors synchronises the handle's streams and returns the bits (0 = none). */
#define CF_GUARD_CELL_BOUNDS 1
#define CF_GUARD_CLUSTER_TABLE 2
#define CF_GUARD_LIST_ENTRY 4
#define CF_GUARD_GRID_BINS 8
#define CF_GUARD_NEIGHBOR 16
#define CF_GUARD_ATOM_INDEX 32   /* cf_compute_openmm: an atom_index entry outside [0, N) */
#define CF_GUARD_REBUILD_FLAG 64 /* the neighbour-list rebuild flag found clear on a handle without a skin */
CF_EXPORT int cf_get_device_errors(cf_handle* h, int32_t* bits);

/*
 * Replaces ReferenceCalcCoulForceKernel::execute (ReferenceCoulKernels.cpp:424-636).
 * Device-resident, asynchronous on the handle's stream:
 *   pos_dev    [N*3] fp64 positions (nm), AoS x,y,z, DEVICE memory
 *   box9       host array, current periodic box vectors (rows) in OpenMM's reduced form
 *              a = (ax,0,0), b = (bx,by,0), c = (cx,cy,cz), |bx|,|cx| <= ax/2, |cy| <= by/2
 *              (triclinic boxes take the all-pairs neighbour list); ignored without PBC
 *   forces_dev [N*3] fp64 DEVICE buffer; forces are ADDED (+=) like the reference
 *              (ReferenceCoulKernels.cpp:426, 455, 585, 630).  Only owned atoms when world_size>1.
 *   energy_dev [1] fp64 DEVICE scalar, OVERWRITTEN with the (partial, per rank) energy.
 * Either output may be NULL.  Energy semantics follow the reference, including its
 * quirk that the self/real-space/exclusion terms are accumulated even without
 * CF_INCLUDE_ENERGY in periodic mode (ReferenceCoulKernels.cpp:507-510, 592, 619).
 */
CF_EXPORT int cf_compute(cf_handle* h, const double* pos_dev, const double* box9, int flags,
                         double* forces_dev, double* energy_dev);

/*
 * The same evaluation on an OpenMM GPU platform's own device buffers, without copies -- the
 * conventions the reference's CUDA platform binds its kernels to (CudaCalcCoulForceKernel::execute,
 * platforms/cuda/src/CudaCoulKernels.cpp:523-600: cu.getPosq(), cu.getAtomIndexArray(),
 * cu.getForce(), cu.getEnergyBuffer(), cu.getPaddedNumAtoms()).  Single rank only.
 *   posq        [N] real4 in the platform's sorted order: posq[s] = (x, y, z, w) of atom
 *               atom_index[s] (nm; w -- the platform's charge slot -- is never read or written).
 *               posq_kind: CF_POSQ_DOUBLE4 (double precision: double4) or CF_POSQ_FLOAT4
 *               (single / mixed precision: float4; posq_correction, if not NULL, is the mixed
 *               platform's float4 posqCorrection, added in fp64)
 *   atom_index  [N] int32 DEVICE array: sorted slot -> atom index (cu.getAtomIndexArray())
 *   padded_n    paddedNumAtoms: the stride of the force planes (>= N)
 *   force_buf   [3 * padded_n] long long DEVICE array, fixed point in units of 2^-32 kJ/mol/nm, the
 *               x, y, z planes one after the other, indexed by sorted slot: forces are ADDED
 *               (OpenMM's conversion (long long)(f * 2^32), 64-bit atomic adds).  NULL: no forces.
 *   energy_buf  DEVICE address of one energy-buffer element (cu.getEnergyBuffer()): the energy
 *               is ADDED to it; energy_kind CF_ENERGY_DOUBLE (mixed / double: `mixed` = double)
 *               or CF_ENERGY_FLOAT (single).  NULL: not written.
 * Energy semantics and flags as cf_compute.  The positions are gathered into the handle's atom
 * order and the forces scattered back by two small kernels on the handle's stream (~2 x 3 us at
 * C3); everything between is cf_compute's device-resident path (graph replay included).
 */
#define CF_POSQ_DOUBLE4 0
#define CF_POSQ_FLOAT4 1
#define CF_ENERGY_DOUBLE 0
#define CF_ENERGY_FLOAT 1
CF_EXPORT int cf_compute_openmm(cf_handle* h, const void* posq, const void* posq_correction, int32_t posq_kind,
                                const int32_t* atom_index, int32_t padded_n, const double* box9, int flags,
                                long long* force_buf, void* energy_buf, int32_t energy_kind);

/* Split-phase form for multi-GPU: begin computes charges and this rank's partial
 * structure factors; the caller all-reduces (sum) the buffer returned by
 * cf_kspace_buffer (fp64, on device, on the handle's stream ordering); end finishes. */
CF_EXPORT int cf_compute_begin(cf_handle* h, const double* pos_dev, const double* box9, int flags);
CF_EXPORT int cf_kspace_buffer(cf_handle* h, double** buf_dev, int64_t* count);
/* Optional, between cf_compute_begin and cf_compute_end: launch the direct-space and
 * exclusion kernels now.  They do not depend on the structure factors, so a multi-rank
 * caller launches them after starting the S(k) all-reduce and before waiting for it (the
 * two overlap).  cf_compute_end runs them itself if this was not called. */
CF_EXPORT int cf_compute_direct(cf_handle* h);
CF_EXPORT int cf_compute_end(cf_handle* h, double* forces_dev, double* energy_dev);

/* Graph replay: enable = 1 captures the launches of an evaluation into hipGraphs (on a private
 * stream) and replays them on the handle's stream while the calls look the same to the host:
 * same device buffers, flags, box and neighbour-list decision (a rebuild under a kept skin is
 * decided on the device, inside the graph).  A change re-captures.  A single-rank cf_compute /
 * cf_compute_host is one graph; the split-phase calls of a multi-rank step are three (begin,
 * direct, end: the caller's all-reduce runs between them on the same stream).  Evaluations with
 * timing on run eagerly.  Results are identical either way (the same kernels in the same order). */
CF_EXPORT int cf_set_graph(cf_handle* h, int enable);
/* Number of graph captures and replays since cf_set_graph(h, 1). */
CF_EXPORT int cf_get_graph_stats(const cf_handle* h, int64_t* captures, int64_t* replays);

/* Second stream (default on; cf_options.handover selects its fork / join): with the
 * grid k-space a single-rank cf_compute runs the reciprocal chain, and the split-phase calls of
 * a multi-rank step run the direct-space chain, on a second stream of the handle, joined before
 * the chain rule.  Results are bitwise those of the one-stream order.  enable = 0 launches
 * everything on the handle's stream (kernel durations are then the kernels' own). */
CF_EXPORT int cf_set_overlap(cf_handle* h, int enable);

/* Synchronous host-memory convenience (H2D positions, D2H forces/energy): what an
 * OpenMM Reference/CPU-platform adapter calls.  forces_host is ADDED to. */
CF_EXPORT int cf_compute_host(cf_handle* h, const double* pos_host, const double* box9, int flags,
                              double* forces_host, double* energy_host);

/* Diagnostics of the last evaluation (synchronous, host outputs).
 *   charges [N]  realcharges after charge flux          (ReferenceCoulKernels.cpp:37-228)
 *   dedq    [N]  dE/dq_i (complete: self+recip+direct+exclusion)
 *   terms   [4]  E_self, E_recip, E_direct(incl. LJ), E_exclusion (PBC); [0,0,E,0] without PBC */
CF_EXPORT int cf_get_charges(cf_handle* h, double* charges_host);
CF_EXPORT int cf_get_dedq(cf_handle* h, double* dedq_host);
CF_EXPORT int cf_get_energy_terms(cf_handle* h, double terms[4]);
CF_EXPORT int cf_synchronize(cf_handle* h);

/* Per-kernel timing: when enabled, start/stop hipEvents are recorded on the handle's
 * stream around every kernel launch of every evaluation (negligible overhead).
 * cf_get_timing synchronises and returns, per phase, the summed milliseconds and the
 * number of recorded launches since cf_set_timing; names are 16-byte NUL-padded. */
CF_EXPORT int cf_set_timing(cf_handle* h, int enable);
/* As cf_set_timing, but only the phases whose bit is set in phase_mask (bit p = the p-th
 * phase name cf_get_timing reports) are bracketed by events; 0 disables timing.  Each timed
 * launch costs two event records on the stream, so a benchmark times only what it reports. */
CF_EXPORT int cf_set_timing_mask(cf_handle* h, uint32_t phase_mask);
CF_EXPORT int cf_get_timing(cf_handle* h, int32_t max_phases, char* names, double* total_ms, int32_t* calls,
                            int32_t* nphases);

#ifdef __cplusplus
}
#endif
#endif /* CHARGEFLUX_H_ */
