// TEST INFRASTRUCTURE ONLY (openmm_compat): the part of OpenMM::Force that CoulForce.h
// (reference: openmmapi/include/CoulForce.h:16, 58, 136) and the plugin use.
#ifndef OPENMM_FORCE_H_
#define OPENMM_FORCE_H_
#include <string>

#include "internal/windowsExport.h"

namespace OpenMM {
class Context;
class ContextImpl;
class ForceImpl;

class OPENMM_EXPORT Force {
public:
    Force() : forceGroup(0) {}
    virtual ~Force() {}
    int getForceGroup() const;
    void setForceGroup(int group);
    const std::string& getName() const;
    void setName(const std::string& name);
    virtual bool usesPeriodicBoundaryConditions() const { return false; }

protected:
    friend class ContextImpl;
    virtual ForceImpl* createImpl() const = 0;

private:
    int forceGroup;
    std::string name;
};
}  // namespace OpenMM
#endif
