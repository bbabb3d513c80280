// HipCoulKernels.h — CalcCoulForceKernel (openmmapi/include/CoulKernels.h:15-38) on MI355X.
//
// Needs OpenMM's headers and the reference's openmmapi/include (CoulForce.h, CoulKernels.h):
// built by plugin/Makefile (`make plugin OPENMM_DIR=... COUL_DIR=...`); in this image it is
// built against the test-only OpenMM compat tree (tests/cpp/openmm_compat, `make compat-plugin`).  Everything the
// kernel does is in coulhip::KernelCore (include/CoulHipKernelCore.h), which is compiled and
// tested without OpenMM through tests/cpp/adapter_capi.cpp.
#ifndef HIP_COUL_KERNELS_H_
#define HIP_COUL_KERNELS_H_

#include <string>

#include "CoulHipKernelCore.h"
#include "CoulKernels.h"
#include "openmm/Platform.h"

namespace CoulPlugin {

class HipCalcCoulForceKernel : public CalcCoulForceKernel {
public:
    // options.one_4pi_eps0 is overwritten with the ONE_4PI_EPS0 of the OpenMM this plugin is
    // built against (HipCoulKernels.cpp)
    HipCalcCoulForceKernel(std::string name, const OpenMM::Platform& platform, const coulhip::Options& options);
    // replaces ReferenceCalcCoulForceKernel::initialize (ReferenceCoulKernels.cpp:230-422)
    void initialize(const OpenMM::System& system, const CoulForce& force) override;
    // replaces ReferenceCalcCoulForceKernel::execute (ReferenceCoulKernels.cpp:424-636)
    double execute(OpenMM::ContextImpl& context, bool includeForces, bool includeEnergy) override;
    // what a CoulForce::updateParametersInContext would call (OpenMM's NonbondedForce pattern;
    // the reference has none)
    void copyParametersToContext(OpenMM::ContextImpl& context, const CoulForce& force);

private:
    coulhip::Options options_;
    coulhip::KernelCore core_;
};

}  // namespace CoulPlugin

#endif  // HIP_COUL_KERNELS_H_
