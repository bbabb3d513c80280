// CoulHipMarshal.h — CoulForce -> cf_params (include/chargeflux.h), header-only.
//
// The OpenMM plugin's initialize() (HipCalcCoulForceKernel, src/HipCoulKernels.cpp) and the
// updateParametersInContext path read the force ONLY through the public getters of
// CoulPlugin::CoulForce, with the reference's exact signatures
// (openmmapi/include/CoulForce.h:37,82,105,117,129), in the order the Reference kernel reads
// them (platforms/reference/src/ReferenceCoulKernels.cpp:230-284 particles and flux terms,
// :385-391 exceptions).  It is a template over the force type so that it compiles both
// against the real CoulForce (built with OpenMM) and against the test-only class
// tests/cpp/CoulForceStandIn.h that has the same getters (built here, where OpenMM is absent).
#ifndef COUL_HIP_MARSHAL_H_
#define COUL_HIP_MARSHAL_H_

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "chargeflux.h"

namespace coulhip {

// The flat storage cf_create / cf_update_parameters read (CoulForce.h:138-149 layout).
struct ForceArrays {
    int32_t num_particles = 0;
    std::vector<double> charges, sigmas, epsilons;          // [N] each
    std::vector<int32_t> exceptions;                        // [2E]
    std::vector<int32_t> bond_idx;    std::vector<double> bond_par;    // [2B], [2B] (k, b)
    std::vector<int32_t> angle_idx;   std::vector<double> angle_par;   // [3A], [2A] (k, theta0)
    std::vector<int32_t> water_idx;   std::vector<double> water_par;   // [3W], [5W] (k1,k2,kub,b0,ub0)
    int32_t use_pbc = 0;
    double cutoff = 1.0, ewald_tol = 1e-4;
    double default_box[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    double one_4pi_eps0 = 0.0;   // the loading OpenMM's ONE_4PI_EPS0 (0 = CF_ONE_4PI_EPS0)

    // cf_params pointing into this object's vectors (valid while it lives, unmodified)
    cf_params params() const {
        cf_params p;
        std::memset(&p, 0, sizeof(p));
        p.num_particles = num_particles;
        p.charges = charges.data();
        p.sigmas = sigmas.data();
        p.epsilons = epsilons.data();
        p.num_exceptions = (int32_t)(exceptions.size() / 2);
        p.exceptions = exceptions.data();
        p.num_flux_bonds = (int32_t)(bond_idx.size() / 2);
        p.flux_bond_idx = bond_idx.data();
        p.flux_bond_params = bond_par.data();
        p.num_flux_angles = (int32_t)(angle_idx.size() / 3);
        p.flux_angle_idx = angle_idx.data();
        p.flux_angle_params = angle_par.data();
        p.num_flux_waters = (int32_t)(water_idx.size() / 3);
        p.flux_water_idx = water_idx.data();
        p.flux_water_params = water_par.data();
        p.use_pbc = use_pbc;
        p.cutoff = cutoff;
        p.ewald_tol = ewald_tol;
        std::memcpy(p.default_box, default_box, sizeof(default_box));
        p.one_4pi_eps0 = one_4pi_eps0;
        return p;
    }
};

// Reads every parameter of `force` through the CoulForce getters.  num_particles is the
// System's particle count (ReferenceCoulKernels.cpp:231 sizes everything by the System);
// default_box = System::getDefaultPeriodicBoxVectors as rows a, b, c (kmax is derived from
// it, ReferenceCoulKernels.cpp:399-420).
template <class ForceT>
ForceArrays marshal(const ForceT& force, int num_particles, const double default_box[9]) {
    if (num_particles != force.getNumParticles())
        throw std::invalid_argument("System and CoulForce have different numbers of particles (" +
                                    std::to_string(num_particles) + " vs " + std::to_string(force.getNumParticles()) +
                                    ")");
    ForceArrays a;
    a.num_particles = num_particles;
    a.charges.resize(num_particles);
    a.sigmas.resize(num_particles);
    a.epsilons.resize(num_particles);
    for (int i = 0; i < num_particles; i++) {   // RCK:233-240
        double q, sig, eps;
        force.getParticleParameters(i, q, sig, eps);
        a.charges[i] = q;
        a.sigmas[i] = sig;
        a.epsilons[i] = eps;
    }
    const int B = force.getNumFluxBonds();      // RCK:242-253
    a.bond_idx.resize(2 * (size_t)B);
    a.bond_par.resize(2 * (size_t)B);
    for (int t = 0; t < B; t++) {
        int p1, p2;
        double k, b;
        force.getFluxBondParameters(t, p1, p2, k, b);
        a.bond_idx[2 * t] = p1; a.bond_idx[2 * t + 1] = p2;
        a.bond_par[2 * t] = k;  a.bond_par[2 * t + 1] = b;
    }
    const int A = force.getNumFluxAngles();     // RCK:255-267, p2 is the central atom
    a.angle_idx.resize(3 * (size_t)A);
    a.angle_par.resize(2 * (size_t)A);
    for (int t = 0; t < A; t++) {
        int p1, p2, p3;
        double k, theta;
        force.getFluxAngleParameters(t, p1, p2, p3, k, theta);
        a.angle_idx[3 * t] = p1; a.angle_idx[3 * t + 1] = p2; a.angle_idx[3 * t + 2] = p3;
        a.angle_par[2 * t] = k;  a.angle_par[2 * t + 1] = theta;
    }
    const int W = force.getNumFluxWaters();     // RCK:269-284
    a.water_idx.resize(3 * (size_t)W);
    a.water_par.resize(5 * (size_t)W);
    for (int t = 0; t < W; t++) {
        int po, ph1, ph2;
        double k1, k2, kub, b0, ub0;
        force.getFluxWaterParameters(t, po, ph1, ph2, k1, k2, kub, b0, ub0);
        a.water_idx[3 * t] = po; a.water_idx[3 * t + 1] = ph1; a.water_idx[3 * t + 2] = ph2;
        double* w = &a.water_par[5 * (size_t)t];
        w[0] = k1; w[1] = k2; w[2] = kub; w[3] = b0; w[4] = ub0;
    }
    const int E = force.getNumExceptions();     // RCK:385-391
    a.exceptions.resize(2 * (size_t)E);
    for (int k = 0; k < E; k++) {
        int p1, p2;
        force.getExceptionParameters(k, p1, p2);
        a.exceptions[2 * k] = p1;
        a.exceptions[2 * k + 1] = p2;
    }
    a.use_pbc = force.usesPeriodicBoundaryConditions() ? 1 : 0;
    a.cutoff = force.getCutoffDistance();
    a.ewald_tol = force.getEwaldErrorTolerance();
    for (int k = 0; k < 9; k++) a.default_box[k] = default_box ? default_box[k] : 0.0;
    return a;
}

}  // namespace coulhip

#endif  // COUL_HIP_MARSHAL_H_
