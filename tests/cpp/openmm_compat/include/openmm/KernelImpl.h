// TEST INFRASTRUCTURE ONLY (openmm_compat): OpenMM::KernelImpl, the base of
// CalcCoulForceKernel (reference: openmmapi/include/CoulKernels.h:15-22).
#ifndef OPENMM_KERNELIMPL_H_
#define OPENMM_KERNELIMPL_H_
#include <string>

#include "internal/windowsExport.h"

namespace OpenMM {
class Platform;

class OPENMM_EXPORT KernelImpl {
public:
    KernelImpl(std::string name, const Platform& platform);
    virtual ~KernelImpl() {}
    std::string getName() const;
    const Platform& getPlatform();

private:
    friend class Kernel;
    std::string name;
    const Platform* platform;
    int referenceCount;
};
}  // namespace OpenMM
#endif
