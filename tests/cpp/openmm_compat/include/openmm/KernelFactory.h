// TEST INFRASTRUCTURE ONLY (openmm_compat): OpenMM::KernelFactory
// (reference: platforms/reference/include/ReferenceCoulKernelFactory.h:13-16).
#ifndef OPENMM_KERNELFACTORY_H_
#define OPENMM_KERNELFACTORY_H_
#include <string>

#include "KernelImpl.h"
#include "internal/windowsExport.h"

namespace OpenMM {
class ContextImpl;

class OPENMM_EXPORT KernelFactory {
public:
    virtual KernelImpl* createKernelImpl(std::string name, const Platform& platform, ContextImpl& context) const = 0;
    virtual ~KernelFactory() {}
};
}  // namespace OpenMM
#endif
