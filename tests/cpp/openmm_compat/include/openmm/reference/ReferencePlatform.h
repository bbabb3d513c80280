// TEST INFRASTRUCTURE ONLY (openmm_compat): OpenMM::ReferencePlatform and its PlatformData,
// whose void* buffers hold a vector<Vec3> of positions and forces and a Vec3[3] of box vectors
// (what ReferenceCoulKernels.cpp:14-27 and the HIP plugin read).  OpenMM's CPU platform derives
// from ReferencePlatform; the compat library registers both.
#ifndef OPENMM_REFERENCEPLATFORM_H_
#define OPENMM_REFERENCEPLATFORM_H_
#include <string>

#include "../Platform.h"
#include "../System.h"
#include "../internal/windowsExport.h"

namespace OpenMM {
class OPENMM_EXPORT ReferencePlatform : public Platform {
public:
    class PlatformData;
    ReferencePlatform();
    const std::string& getName() const {
        static const std::string name = "Reference";
        return name;
    }
    double getSpeed() const { return 1; }
    bool supportsDoublePrecision() const { return true; }
};

class OPENMM_EXPORT ReferencePlatform::PlatformData {
public:
    PlatformData(const System& system);
    ~PlatformData();
    int numParticles, stepCount;
    double time;
    void* positions;
    void* velocities;
    void* forces;
    void* periodicBoxSize;
    void* periodicBoxVectors;
};
}  // namespace OpenMM
#endif
