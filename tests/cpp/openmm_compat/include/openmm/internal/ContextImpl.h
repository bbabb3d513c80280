// TEST INFRASTRUCTURE ONLY (openmm_compat): OpenMM::ContextImpl reduced to what kernels use
// (getPlatform, getPlatformData).  In OpenMM a Context creates it; here the test host builds
// one directly around a ReferencePlatform::PlatformData.
#ifndef OPENMM_CONTEXTIMPL_H_
#define OPENMM_CONTEXTIMPL_H_
#include "../internal/windowsExport.h"

namespace OpenMM {
class Platform;

class OPENMM_EXPORT ContextImpl {
public:
    ContextImpl(Platform& platform, void* platformData) : platform(&platform), platformData(platformData) {}
    Platform& getPlatform() { return *platform; }
    void* getPlatformData() { return platformData; }
    const void* getPlatformData() const { return platformData; }
    void setPlatformData(void* data) { platformData = data; }

private:
    Platform* platform;
    void* platformData;
};
}  // namespace OpenMM
#endif
