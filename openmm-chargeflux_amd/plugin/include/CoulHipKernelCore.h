// CoulHipKernelCore.h — the OpenMM-independent body of HipCalcCoulForceKernel.
//
// Owns one cf_handle (include/chargeflux.h) and implements what the kernel interface asks for
// (openmmapi/include/CoulKernels.h:15-38): initialize from a System's particle count + default
// box and a CoulForce, execute with includeForces / includeEnergy returning the energy and
// ADDING forces (ReferenceCoulKernels.cpp:424-636), and the parameter update that
// updateParametersInContext would route here.  Errors become coulhip::Error (the OpenMM layer
// rethrows them as OpenMMException, like every OpenMM kernel; SURVEY §8(b) "Errors").
// Header-only so the OpenMM plugin (src/HipCoulKernels.cpp) and the test library
// (tests/cpp/adapter_capi.cpp) compile the same code.
#ifndef COUL_HIP_KERNEL_CORE_H_
#define COUL_HIP_KERNEL_CORE_H_

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "CoulHipMarshal.h"
#include "chargeflux.h"

namespace coulhip {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

inline void check(int rc, const char* what) {
    if (rc != CF_OK) throw Error(rc, std::string(what) + ": " + cf_last_error());
}

// cf_options in plugin terms.  Defaults: device 0, the null stream, one rank, fp64, the grid
// reciprocal path (kspace_algo 2, the benchmarked one; 0 = exact fp64-MFMA k-sum).
struct Options {
    int device = 0;
    void* stream = nullptr;
    int kspace_algo = 2;
    int grid_width = 0;
    int precision = CF_PRECISION_DOUBLE;   // OpenMM platform property "Precision": "double" / "mixed"
    int rank = 0, world_size = 1;
    double neighbor_skin = 0.0;            // nm; 0 = rebuild every call like the reference
    // ONE_4PI_EPS0 of the OpenMM this kernel is loaded into (the reference compiles it in from
    // openmm/reference/SimTKOpenMMRealType.h, ReferenceCoulKernels.cpp:7; the plugin's OpenMM layer
    // sets it the same way, src/HipCoulKernels.cpp).  0 = CF_ONE_4PI_EPS0 (OpenMM 7.x).
    double one_4pi_eps0 = 0.0;
};

class KernelCore {
public:
    KernelCore() = default;
    KernelCore(const KernelCore&) = delete;
    KernelCore& operator=(const KernelCore&) = delete;
    ~KernelCore() { release(); }

    // ReferenceCalcCoulForceKernel::initialize (ReferenceCoulKernels.cpp:230-422)
    template <class ForceT>
    void initialize(const ForceT& force, int num_particles, const double default_box[9], const Options& o) {
        ForceArrays a = marshal(force, num_particles, default_box);
        a.one_4pi_eps0 = o.one_4pi_eps0;
        cf_params p = a.params();
        cf_options opt;
        std::memset(&opt, 0, sizeof(opt));
        opt.device = o.device;
        opt.stream = o.stream;
        opt.rank = o.rank;
        opt.world_size = o.world_size;
        opt.kspace_algo = o.kspace_algo;
        opt.grid_width = o.grid_width;
        opt.precision = o.precision;
        release();
        check(cf_create(&p, &opt, &h_), "cf_create");
        if (o.neighbor_skin > 0) check(cf_set_neighbor_skin(h_, o.neighbor_skin), "cf_set_neighbor_skin");
        n_ = num_particles;
        pbc_ = a.use_pbc != 0;
        ke_ = o.one_4pi_eps0;
    }

    // updateParametersInContext -> copyParametersToContext (the reference has none):
    // the same getters, then cf_update_parameters (topology must be unchanged)
    template <class ForceT>
    void copy_parameters(const ForceT& force) {
        require();
        ForceArrays a = marshal(force, n_, nullptr);
        a.one_4pi_eps0 = ke_;
        cf_params p = a.params();
        check(cf_update_parameters(h_, &p), "cf_update_parameters");
    }

    // ReferenceCalcCoulForceKernel::execute on host arrays (the Reference/CPU platforms'
    // vector<Vec3> storage is three contiguous doubles per particle): forces are ADDED.
    double execute_host(const double* pos, const double* box9, bool include_forces, bool include_energy,
                        double* forces_accum) {
        require();
        double e = 0.0;
        check(cf_compute_host(h_, pos, pbc_ ? box9 : nullptr, flags(include_forces, include_energy), forces_accum, &e),
              "cf_compute_host");
        watch_fallbacks();   // (the host path has synchronised: one small read)
        return e;
    }

    // an OpenMM GPU platform's own buffers (cf_compute_openmm: posq + atomIndex in, 2^32 fixed-point
    // force planes and an energy-buffer element out -- the conventions the reference's CUDA
    // platform binds, CudaCoulKernels.cpp:523-600); asynchronous on the handle's stream
    void execute_openmm(const void* posq, const void* posq_correction, int posq_kind, const int* atom_index,
                        int padded_n, const double* box9, bool include_forces, bool include_energy,
                        long long* force_buf, void* energy_buf, int energy_kind) {
        require();
        check(cf_compute_openmm(h_, posq, posq_correction, posq_kind, atom_index, padded_n, pbc_ ? box9 : nullptr,
                                flags(include_forces, include_energy), force_buf, energy_buf, energy_kind),
              "cf_compute_openmm");
        if (++device_calls_ % kFallbackPoll == 0) watch_fallbacks();   // (synchronises: amortised)
    }

    // the same on device buffers (a HIP platform's positions / forces): asynchronous on the stream
    void execute_device(const double* pos_dev, const double* box9, bool include_forces, bool include_energy,
                        double* forces_dev, double* energy_dev) {
        require();
        check(cf_compute(h_, pos_dev, pbc_ ? box9 : nullptr, flags(include_forces, include_energy), forces_dev,
                         energy_dev),
              "cf_compute");
        if (++device_calls_ % kFallbackPoll == 0) watch_fallbacks();
    }

    cf_handle* handle() const { return h_; }
    int num_particles() const { return n_; }

    // Evaluations that fell back to the fp64 cell rescan (cf_get_fallback_stats: a neighbour list
    // or window that overflowed, a term beyond the fixed-point range) -- correct, several times
    // slower.  The first one seen is reported once on stderr (COUL_HIP_QUIET=1 silences it); this
    // counter stays readable.
    long long fallback_evaluations() {
        watch_fallbacks();
        return fallbacks_;
    }

private:
    static int flags(bool f, bool e) { return (f ? CF_INCLUDE_FORCES : 0) | (e ? CF_INCLUDE_ENERGY : 0); }
    void require() const {
        if (!h_) throw Error(CF_ERR_STATE, "the kernel has not been initialized");
    }
    void release() {
        if (h_) cf_destroy(h_);
        h_ = nullptr;
    }
    static constexpr long long kFallbackPoll = 1000;   // device-path calls between checks
    void watch_fallbacks() {
        if (!h_) return;
        int64_t evals = 0, rows = 0;
        int32_t reasons = 0;
        if (cf_get_fallback_stats(h_, &evals, &rows, &reasons) != CF_OK) return;
        const long long total = (long long)evals + (long long)rows;
        if (total > fallbacks_ && !warned_) {
            warned_ = true;
            const char* quiet = std::getenv("COUL_HIP_QUIET");
            if (!quiet || quiet[0] != '1')
                std::fprintf(stderr,
                             "CoulForce (HIP): %lld evaluation(s) took the fp64 rescan fallback and %lld list row(s) "
                             "were rescanned (reasons 0x%x: 1 = cell window full, 2 = list overflow, 4 = fixed-point "
                             "range) -- correct but slow; check the neighbour-list capacity and cell geometry "
                             "(DESIGN.md 4.4). Reported once.\n",
                             (long long)evals, (long long)rows, (unsigned)reasons);
        }
        fallbacks_ = total;
    }
    cf_handle* h_ = nullptr;
    int n_ = 0;
    bool pbc_ = false;
    double ke_ = 0.0;
    long long device_calls_ = 0, fallbacks_ = 0;
    bool warned_ = false;
};

}  // namespace coulhip

#endif  // COUL_HIP_KERNEL_CORE_H_
