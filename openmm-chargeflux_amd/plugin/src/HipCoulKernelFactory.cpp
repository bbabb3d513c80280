// HipCoulKernelFactory.cpp — OpenMM plugin registration of the MI355X CoulForce kernel.
//
// OpenMM dlopen()s lib/plugins/*.so and calls the two extern "C" entry points below; the
// third is the explicit registration call, like registerCoulReferenceKernelFactories /
// registerCoulCudaKernelFactories (platforms/reference/src/ReferenceCoulKernelFactory.cpp:12-36,
// platforms/cuda/src/CudaCoulKernelFactory.cpp:13-44).  The factory attaches to every platform
// whose contexts carry ReferencePlatform::PlatformData (Reference, and CPU, which derives from
// it), where HipCalcCoulForceKernel moves positions in and forces out per step through
// cf_compute_host.
//
// Options (OpenMM's Reference and CPU platforms have no property a plugin may add, so they are
// environment variables, read when a kernel is created):
//   COUL_HIP_KSPACE     "exact" (fp64-MFMA k-sum) or "grid"; default: exact on the platform
//                       named "Reference" (reference semantics), grid elsewhere
//   COUL_HIP_PRECISION  "double" (default) or "mixed"
//   COUL_HIP_DEVICE     HIP device ordinal (default 0)
//   COUL_HIP_SKIN       neighbour-list skin in nm (default 0: rebuild every call, as the reference)
//   COUL_HIP_YIELD      "1": leave a platform alone when another CalcCoulForce factory (e.g. the
//                       reference's libOpenMMCoulReference) is already registered on it
//
// Both this library and the reference's libOpenMMCoulReference register "CalcCoulForce" on the
// Reference/CPU platforms, and OpenMM keeps the LAST registration.  registerKernelFactories
// detects a factory that is already there (Platform::supportsKernels), replaces it unless
// COUL_HIP_YIELD=1, and says so on stderr; coulHipRegistrationReport() returns the same record.
// If the reference library registers after this one it wins instead; calling
// registerCoulHipKernelFactories() after loading the plugins makes the HIP kernel the winner.
// The XML serialization proxy of CoulForce (CoulForceProxy.cpp) is registered here too.
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <string>
#include <typeinfo>

#include "CoulForceProxy.h"
#include "HipCoulKernels.h"
#include "openmm/KernelFactory.h"
#include "openmm/OpenMMException.h"
#include "openmm/internal/ContextImpl.h"
#include "openmm/reference/ReferencePlatform.h"
#include "openmm/serialization/SerializationProxy.h"

using namespace CoulPlugin;
using namespace OpenMM;

namespace CoulPlugin {

class HipCoulKernelFactory : public KernelFactory {
public:
    KernelImpl* createKernelImpl(std::string name, const Platform& platform, ContextImpl& context) const override {
        if (name != CalcCoulForceKernel::Name())
            throw OpenMMException("Tried to create kernel with illegal kernel name '" + name + "'");
        (void)context;
        return new HipCalcCoulForceKernel(name, platform, options_for(platform.getName()));
    }

    static coulhip::Options options_for(const std::string& platform_name) {
        coulhip::Options o;
        // the Reference platform promises reference semantics: the exact k-sum by default
        o.kspace_algo = platform_name == "Reference" ? 0 : 2;
        const char* ks = std::getenv("COUL_HIP_KSPACE");
        if (ks && std::string(ks) == "exact") o.kspace_algo = 0;
        if (ks && std::string(ks) == "grid") o.kspace_algo = 2;
        const char* prec = std::getenv("COUL_HIP_PRECISION");
        if (prec && std::string(prec) == "mixed") o.precision = CF_PRECISION_MIXED;
        const char* dev = std::getenv("COUL_HIP_DEVICE");
        if (dev) o.device = std::atoi(dev);
        const char* skin = std::getenv("COUL_HIP_SKIN");
        if (skin) o.neighbor_skin = std::atof(skin);
        return o;
    }
};

}  // namespace CoulPlugin

namespace {
std::string g_report;   // one line per platform visited by the last registerKernelFactories()
}

extern "C" OPENMM_EXPORT void registerPlatforms() {}

extern "C" OPENMM_EXPORT void registerKernelFactories() {
    static const CoulForceProxy proxy;
    SerializationProxy::registerProxy(typeid(CoulForce), &proxy);
    const char* yield_env = std::getenv("COUL_HIP_YIELD");
    const bool yield = yield_env && std::string(yield_env) == "1";
    g_report.clear();
    for (int i = 0; i < Platform::getNumPlatforms(); i++) {
        Platform& platform = Platform::getPlatform(i);
        if (dynamic_cast<ReferencePlatform*>(&platform) == nullptr) continue;
        const bool taken = platform.supportsKernels({CalcCoulForceKernel::Name()});
        std::string line = platform.getName() + ": ";
        if (taken && yield) {
            line += "kept the CalcCoulForce factory already registered (COUL_HIP_YIELD=1)";
        } else {
            try {
                platform.registerKernelFactory(CalcCoulForceKernel::Name(), new HipCoulKernelFactory());
                line += taken ? "replaced an already registered CalcCoulForce factory with the HIP kernel"
                              : "registered the HIP kernel";
            } catch (const std::exception& e) {
                line += std::string("registration refused (") + e.what() + ")";
            }
        }
        if (taken) std::fprintf(stderr, "libOpenMMCoulHIP: %s\n", line.c_str());
        g_report += line + "\n";
    }
}

extern "C" OPENMM_EXPORT void registerCoulHipKernelFactories() { registerKernelFactories(); }

// What the last registration did on each Reference-derived platform (diagnostics).
extern "C" OPENMM_EXPORT const char* coulHipRegistrationReport() { return g_report.c_str(); }
