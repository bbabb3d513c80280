// TEST INFRASTRUCTURE ONLY (openmm_compat): OpenMM::Kernel, the reference-counted handle
// Platform::createKernel returns (CoulForceImpl.cpp:25 calls getAs<CalcCoulForceKernel>()).
#ifndef OPENMM_KERNEL_H_
#define OPENMM_KERNEL_H_
#include <string>

#include "KernelImpl.h"
#include "OpenMMException.h"
#include "internal/windowsExport.h"

namespace OpenMM {
class OPENMM_EXPORT Kernel {
public:
    Kernel();
    Kernel(KernelImpl* impl);
    Kernel(const Kernel& copy);
    ~Kernel();
    Kernel& operator=(const Kernel& copy);
    std::string getName() const;
    const KernelImpl& getImpl() const;
    KernelImpl& getImpl();
    template <class T>
    T& getAs() {
        return dynamic_cast<T&>(*impl);
    }

private:
    KernelImpl* impl;
};
}  // namespace OpenMM
#endif
