// HipCoulKernels.cpp — OpenMM glue of HipCalcCoulForceKernel (see HipCoulKernels.h).
//
// Positions, forces and box come from the host platform's data the same way the Reference
// kernel reads them (ReferenceCoulKernels.cpp:14-27): a ReferencePlatform::PlatformData whose
// vector<Vec3> buffers are three contiguous doubles per particle, so they cross the C-ABI as
// [N*3] arrays; forces are ADDED (cf_compute_host), the energy is returned.  The Coulomb
// constant is the ONE_4PI_EPS0 of the OpenMM this file is compiled against -- the header the
// reference itself takes it from (ReferenceCoulKernels.cpp:7) -- so the two agree whatever the
// OpenMM version (138.935456 in 7.x, 138.93545764438198 in 8.x).
#include "HipCoulKernels.h"

#include <vector>

#include "openmm/OpenMMException.h"
#include "openmm/System.h"
#include "openmm/Vec3.h"
#include "openmm/internal/ContextImpl.h"
#include "openmm/reference/ReferencePlatform.h"
#include "openmm/reference/SimTKOpenMMRealType.h"

using namespace CoulPlugin;
using namespace OpenMM;

static_assert(sizeof(Vec3) == 3 * sizeof(double), "Vec3 must be three packed doubles to cross the C-ABI");

namespace {

ReferencePlatform::PlatformData* platform_data(ContextImpl& context) {
    return reinterpret_cast<ReferencePlatform::PlatformData*>(context.getPlatformData());
}

template <class F>
auto rethrow(F&& f) -> decltype(f()) {
    try {
        return f();
    } catch (const coulhip::Error& e) {
        throw OpenMMException(e.what());
    } catch (const std::invalid_argument& e) {
        throw OpenMMException(e.what());
    }
}

}  // namespace

HipCalcCoulForceKernel::HipCalcCoulForceKernel(std::string name, const Platform& platform,
                                               const coulhip::Options& options)
    : CalcCoulForceKernel(name, platform), options_(options) {
    options_.one_4pi_eps0 = ONE_4PI_EPS0;
}

void HipCalcCoulForceKernel::initialize(const System& system, const CoulForce& force) {
    Vec3 a, b, c;
    system.getDefaultPeriodicBoxVectors(a, b, c);   // kmax from the default box (RCK:399-420)
    const double box[9] = {a[0], a[1], a[2], b[0], b[1], b[2], c[0], c[1], c[2]};
    rethrow([&] { core_.initialize(force, system.getNumParticles(), box, options_); });
}

double HipCalcCoulForceKernel::execute(ContextImpl& context, bool includeForces, bool includeEnergy) {
    ReferencePlatform::PlatformData* data = platform_data(context);
    std::vector<Vec3>& pos = *reinterpret_cast<std::vector<Vec3>*>(data->positions);
    std::vector<Vec3>& frc = *reinterpret_cast<std::vector<Vec3>*>(data->forces);
    const Vec3* bv = reinterpret_cast<const Vec3*>(data->periodicBoxVectors);
    const double box[9] = {bv[0][0], bv[0][1], bv[0][2], bv[1][0], bv[1][1], bv[1][2], bv[2][0], bv[2][1], bv[2][2]};
    return rethrow([&] {
        return core_.execute_host(&pos[0][0], box, includeForces, includeEnergy, &frc[0][0]);
    });
}

void HipCalcCoulForceKernel::copyParametersToContext(ContextImpl&, const CoulForce& force) {
    rethrow([&] { core_.copy_parameters(force); });
}
