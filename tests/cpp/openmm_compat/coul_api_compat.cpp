// TEST INFRASTRUCTURE ONLY — libOpenMMCoul.so of the openmm_compat tree: member definitions
// for the reference's own class declaration CoulPlugin::CoulForce (compiled against
// /root/reference/openmmapi/include/CoulForce.h, read in place), so the plugin can be linked
// and driven here.  The reference builds this library from openmmapi/src/CoulForce.cpp with
// OpenMM; that file is not used.  Same observable behaviour through the public API (defaults
// cutoff 1.0 nm, Ewald tolerance 1e-4, no PBC: CoulForce.cpp:12-16); out-of-range indices
// throw OpenMMException here.  createImpl() needs OpenMM's ForceImpl machinery and throws.
#include <string>

#include "CoulForce.h"
#include "openmm/OpenMMException.h"

using CoulPlugin::CoulForce;

namespace {
void check_index(int index, size_t count, const char* what) {
    if (index < 0 || (size_t)index >= count)
        throw OpenMM::OpenMMException(std::string(what) + " index " + std::to_string(index) + " out of range");
}
}  // namespace

CoulForce::CoulForce() : cutoffDistance(1.0), ewaldTol(1e-4), ifPBC(false) {}

// particles: charge in `charges`, (sigma, epsilon) interleaved in `ljparams`
void CoulForce::addParticle(double charge, double sigma, double epsilon) {
    charges.push_back(charge);
    ljparams.insert(ljparams.end(), {sigma, epsilon});
}
int CoulForce::getNumParticles() const { return (int)charges.size(); }
void CoulForce::getParticleParameters(int index, double& charge, double& sigma, double& epsilon) const {
    check_index(index, charges.size(), "particle");
    charge = charges[index];
    sigma = ljparams[2 * (size_t)index];
    epsilon = ljparams[2 * (size_t)index + 1];
}
void CoulForce::setParticleParameters(int index, double charge, double sigma, double epsilon) {
    check_index(index, charges.size(), "particle");
    charges[index] = charge;
    ljparams[2 * (size_t)index] = sigma;
    ljparams[2 * (size_t)index + 1] = epsilon;
}

double CoulForce::getCutoffDistance() const { return cutoffDistance; }
void CoulForce::setCutoffDistance(double cutoff) { cutoffDistance = cutoff; }
bool CoulForce::usesPeriodicBoundaryConditions() const { return ifPBC; }
void CoulForce::setUsesPeriodicBoundaryConditions(bool ifPeriod) { ifPBC = ifPeriod; }
void CoulForce::setEwaldErrorTolerance(double tol) { ewaldTol = tol; }
double CoulForce::getEwaldErrorTolerance() const { return ewaldTol; }

void CoulForce::addException(int p1, int p2) { exclusions.emplace_back(p1, p2); }
int CoulForce::getNumExceptions() const { return (int)exclusions.size(); }
void CoulForce::getExceptionParameters(const int index, int& p1, int& p2) const {
    check_index(index, exclusions.size(), "exception");
    p1 = exclusions[index].first;
    p2 = exclusions[index].second;
}

// flux terms: index tuples and parameter tuples in flat vectors, strides 2/2, 3/2, 3/5
void CoulForce::addFluxBond(int p1, int p2, double k, double b) {
    fbond_idx.insert(fbond_idx.end(), {p1, p2});
    fbond_params.insert(fbond_params.end(), {k, b});
}
int CoulForce::getNumFluxBonds() const { return (int)(fbond_idx.size() / 2); }
void CoulForce::getFluxBondParameters(int index, int& p1, int& p2, double& k, double& b) const {
    check_index(index, fbond_idx.size() / 2, "flux bond");
    const size_t t = (size_t)index;
    p1 = fbond_idx[2 * t]; p2 = fbond_idx[2 * t + 1];
    k = fbond_params[2 * t]; b = fbond_params[2 * t + 1];
}
void CoulForce::addFluxAngle(int p1, int p2, int p3, double k, double theta) {
    fangle_idx.insert(fangle_idx.end(), {p1, p2, p3});
    fangle_params.insert(fangle_params.end(), {k, theta});
}
int CoulForce::getNumFluxAngles() const { return (int)(fangle_idx.size() / 3); }
void CoulForce::getFluxAngleParameters(int index, int& p1, int& p2, int& p3, double& k, double& theta) const {
    check_index(index, fangle_idx.size() / 3, "flux angle");
    const size_t t = (size_t)index;
    p1 = fangle_idx[3 * t]; p2 = fangle_idx[3 * t + 1]; p3 = fangle_idx[3 * t + 2];
    k = fangle_params[2 * t]; theta = fangle_params[2 * t + 1];
}
void CoulForce::addFluxWater(int po, int ph1, int ph2, double k1, double k2, double kub, double b0, double ub0) {
    fwater_idx.insert(fwater_idx.end(), {po, ph1, ph2});
    fwater_params.insert(fwater_params.end(), {k1, k2, kub, b0, ub0});
}
int CoulForce::getNumFluxWaters() const { return (int)(fwater_idx.size() / 3); }
void CoulForce::getFluxWaterParameters(int index, int& po, int& ph1, int& ph2, double& k1, double& k2, double& kub,
                                       double& b0, double& ub0) const {
    check_index(index, fwater_idx.size() / 3, "flux water");
    const size_t t = (size_t)index;
    po = fwater_idx[3 * t]; ph1 = fwater_idx[3 * t + 1]; ph2 = fwater_idx[3 * t + 2];
    const double* p = &fwater_params[5 * t];
    k1 = p[0]; k2 = p[1]; kub = p[2]; b0 = p[3]; ub0 = p[4];
}

OpenMM::ForceImpl* CoulForce::createImpl() const {
    throw OpenMM::OpenMMException("CoulForce::createImpl is not available in the openmm_compat test build");
}
