// HipCoulKernelFactory.cpp — OpenMM plugin registration of the MI355X CoulForce kernel.
//
// OpenMM dlopen()s lib/plugins/*.so and calls the two extern "C" entry points below; the
// third is the explicit registration call, like registerCoulReferenceKernelFactories /
// registerCoulCudaKernelFactories (platforms/reference/src/ReferenceCoulKernelFactory.cpp:12-36,
// platforms/cuda/src/CudaCoulKernelFactory.cpp:13-44).  The factory attaches to every platform
// whose contexts carry ReferencePlatform::PlatformData (Reference, and CPU, which derives from
// it), where HipCalcCoulForceKernel moves positions in and forces out per step through
// cf_compute_host; the environment variables COUL_HIP_PRECISION ("double" / "mixed"),
// COUL_HIP_KSPACE ("grid" / "exact") and COUL_HIP_DEVICE select cf_options.  Built only with
// OpenMM (plugin/Makefile).
#include <cstdlib>
#include <exception>
#include <string>

#include "HipCoulKernels.h"
#include "openmm/KernelFactory.h"
#include "openmm/OpenMMException.h"
#include "openmm/internal/ContextImpl.h"
#include "openmm/reference/ReferencePlatform.h"

using namespace CoulPlugin;
using namespace OpenMM;

namespace CoulPlugin {

class HipCoulKernelFactory : public KernelFactory {
public:
    KernelImpl* createKernelImpl(std::string name, const Platform& platform, ContextImpl& context) const override {
        if (name != CalcCoulForceKernel::Name())
            throw OpenMMException("Tried to create kernel with illegal kernel name '" + name + "'");
        coulhip::Options o;
        const char* prec = std::getenv("COUL_HIP_PRECISION");
        if (prec && std::string(prec) == "mixed") o.precision = CF_PRECISION_MIXED;
        const char* ks = std::getenv("COUL_HIP_KSPACE");
        if (ks && std::string(ks) == "exact") o.kspace_algo = 0;
        const char* dev = std::getenv("COUL_HIP_DEVICE");
        if (dev) o.device = std::atoi(dev);
        (void)context;
        return new HipCalcCoulForceKernel(name, platform, o);
    }
};

}  // namespace CoulPlugin

extern "C" OPENMM_EXPORT void registerPlatforms() {}

extern "C" OPENMM_EXPORT void registerKernelFactories() {
    for (int i = 0; i < Platform::getNumPlatforms(); i++) {
        Platform& platform = Platform::getPlatform(i);
        if (dynamic_cast<ReferencePlatform*>(&platform) != nullptr) {
            try {
                platform.registerKernelFactory(CalcCoulForceKernel::Name(), new HipCoulKernelFactory());
            } catch (const std::exception&) {
                // a platform that refuses the factory keeps its own CoulForce kernel (if any)
            }
        }
    }
}

extern "C" OPENMM_EXPORT void registerCoulHipKernelFactories() { registerKernelFactories(); }
