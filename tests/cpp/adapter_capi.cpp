// TEST INFRASTRUCTURE ONLY — libcf_adapter_test.so: drives the OpenMM plugin's C++ layer
// (plugin/include/CoulHipMarshal.h + CoulHipKernelCore.h, the code HipCalcCoulForceKernel runs)
// from Python.  A CoulForce (tests/cpp/CoulForceStandIn.h, the reference's API) is filled
// through its add* setters from flat arrays, exactly as a user's C++ would build it; the
// plugin layer then reads it back through the getters.
//   cfa_marshal : force -> coulhip::ForceArrays, copied out (CPU test: compared with the
//                 Python mirror's cf_params, i.e. the flux-term order the reference reads)
//   cfa_execute : force -> KernelCore::initialize (cf_create) -> execute_host (GPU test:
//                 compared with the oracle), optionally a parameter update in between
#include <cstring>
#include <exception>
#include <string>

#include "CoulForceStandIn.h"
#include "CoulHipKernelCore.h"

namespace {

thread_local std::string g_err;

struct Flat {   // the same layout as the Python mirror's CoulForce.arrays()
    int n;
    const double *q, *sig, *eps;
    int ne;
    const int* ex;
    int nb;
    const int* bi;
    const double* bp;
    int na;
    const int* ai;
    const double* ap;
    int nw;
    const int* wi;
    const double* wp;
    int pbc;
    double cutoff, tol;
};

CoulPlugin::CoulForce build(const Flat& f) {
    CoulPlugin::CoulForce force;
    for (int i = 0; i < f.n; i++) force.addParticle(f.q[i], f.sig[i], f.eps[i]);
    for (int k = 0; k < f.ne; k++) force.addException(f.ex[2 * k], f.ex[2 * k + 1]);
    for (int t = 0; t < f.nb; t++) force.addFluxBond(f.bi[2 * t], f.bi[2 * t + 1], f.bp[2 * t], f.bp[2 * t + 1]);
    for (int t = 0; t < f.na; t++)
        force.addFluxAngle(f.ai[3 * t], f.ai[3 * t + 1], f.ai[3 * t + 2], f.ap[2 * t], f.ap[2 * t + 1]);
    for (int t = 0; t < f.nw; t++) {
        const double* p = f.wp + 5 * t;
        force.addFluxWater(f.wi[3 * t], f.wi[3 * t + 1], f.wi[3 * t + 2], p[0], p[1], p[2], p[3], p[4]);
    }
    force.setUsesPeriodicBoundaryConditions(f.pbc != 0);
    force.setCutoffDistance(f.cutoff);
    force.setEwaldErrorTolerance(f.tol);
    return force;
}

template <class F>
int guarded(F&& fn) {
    try {
        fn();
        return 0;
    } catch (const coulhip::Error& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::exception& e) {
        g_err = e.what();
        return CF_ERR_INVALID;
    }
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) const char* cfa_last_error(void) { return g_err.c_str(); }

// Marshal (for a System of n_system particles) and copy out: q/sig/eps [N], ex [2E], bonds
// [2B]+[2B], angles [3A]+[2A], waters [3W]+[5W], scal = {use_pbc, cutoff, tol}, box_out [9]
__attribute__((visibility("default"))) int cfa_marshal(const Flat* f, int n_system, const double* box9, double* q, double* sig,
                                                       double* eps, int* ex, int* bi, double* bp, int* ai, double* ap,
                                                       int* wi, double* wp, double* scal, double* box_out) {
    return guarded([&] {
        CoulPlugin::CoulForce force = build(*f);
        coulhip::ForceArrays a = coulhip::marshal(force, n_system, box9);
        const cf_params p = a.params();
        std::memcpy(q, p.charges, sizeof(double) * p.num_particles);
        std::memcpy(sig, p.sigmas, sizeof(double) * p.num_particles);
        std::memcpy(eps, p.epsilons, sizeof(double) * p.num_particles);
        std::memcpy(ex, p.exceptions, sizeof(int) * 2 * p.num_exceptions);
        std::memcpy(bi, p.flux_bond_idx, sizeof(int) * 2 * p.num_flux_bonds);
        std::memcpy(bp, p.flux_bond_params, sizeof(double) * 2 * p.num_flux_bonds);
        std::memcpy(ai, p.flux_angle_idx, sizeof(int) * 3 * p.num_flux_angles);
        std::memcpy(ap, p.flux_angle_params, sizeof(double) * 2 * p.num_flux_angles);
        std::memcpy(wi, p.flux_water_idx, sizeof(int) * 3 * p.num_flux_waters);
        std::memcpy(wp, p.flux_water_params, sizeof(double) * 5 * p.num_flux_waters);
        scal[0] = p.use_pbc;
        scal[1] = p.cutoff;
        scal[2] = p.ewald_tol;
        std::memcpy(box_out, p.default_box, sizeof(double) * 9);
    });
}

// Initialize on f, optionally update to the parameters of f2 (same topology), then execute
// once on host arrays.  forces is ADDED to; *energy = the energy.
__attribute__((visibility("default"))) int cfa_execute(const Flat* f, const Flat* f2, const double* default_box,
                                                       int kspace_algo, int precision, const double* pos,
                                                       const double* box9, int include_forces, int include_energy,
                                                       double* forces, double* energy) {
    return guarded([&] {
        CoulPlugin::CoulForce force = build(*f);
        coulhip::Options o;
        o.kspace_algo = kspace_algo;
        o.precision = precision;
        coulhip::KernelCore core;
        core.initialize(force, f->n, default_box, o);
        if (f2) core.copy_parameters(build(*f2));
        *energy = core.execute_host(pos, box9, include_forces != 0, include_energy != 0, forces);
    });
}

// Initialize on f and execute `calls` times on host arrays; *fallbacks = KernelCore::fallback_evaluations()
// (the plugin's slow-path counter; its first increase is reported once on stderr)
__attribute__((visibility("default"))) int cfa_execute_count(const Flat* f, const double* default_box, int kspace_algo,
                                                             const double* pos, const double* box9, int calls,
                                                             double* forces, double* energy, long long* fallbacks) {
    return guarded([&] {
        CoulPlugin::CoulForce force = build(*f);
        coulhip::Options o;
        o.kspace_algo = kspace_algo;
        coulhip::KernelCore core;
        core.initialize(force, f->n, default_box, o);
        for (int c = 0; c < calls; c++) *energy = core.execute_host(pos, box9, true, true, forces);
        *fallbacks = core.fallback_evaluations();
    });
}

}  // extern "C"
