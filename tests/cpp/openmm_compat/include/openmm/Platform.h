// TEST INFRASTRUCTURE ONLY (openmm_compat): the part of OpenMM::Platform a plugin touches --
// the static platform registry (getNumPlatforms / getPlatform / getPlatformByName /
// registerPlatform), registerKernelFactory, supportsKernels and createKernel -- with OpenMM's
// signatures.  As in OpenMM, a later registerKernelFactory for the same name replaces the
// earlier factory.
#ifndef OPENMM_PLATFORM_H_
#define OPENMM_PLATFORM_H_
#include <map>
#include <string>
#include <vector>

#include "Kernel.h"
#include "internal/windowsExport.h"

namespace OpenMM {
class ContextImpl;
class KernelFactory;

class OPENMM_EXPORT Platform {
public:
    virtual ~Platform();
    virtual const std::string& getName() const = 0;
    virtual double getSpeed() const = 0;
    virtual bool supportsDoublePrecision() const = 0;
    const std::vector<std::string>& getPropertyNames() const { return platformProperties; }
    void registerKernelFactory(const std::string& name, KernelFactory* factory);
    bool supportsKernels(const std::vector<std::string>& kernelNames) const;
    Kernel createKernel(const std::string& name, ContextImpl& context) const;
    static void registerPlatform(Platform* platform);
    static int getNumPlatforms();
    static Platform& getPlatform(int index);
    static Platform& getPlatformByName(const std::string& name);

protected:
    std::vector<std::string> platformProperties;

private:
    friend struct CompatRegistryAccess;   // compat only: lets the test host reach a registered factory
    std::map<std::string, KernelFactory*> kernelFactories;
};
}  // namespace OpenMM
#endif
