// TEST INFRASTRUCTURE ONLY (openmm_compat): OpenMM::System (particle masses, forces owned by
// the System, default periodic box) with OpenMM's signatures.
#ifndef OPENMM_SYSTEM_H_
#define OPENMM_SYSTEM_H_
#include <vector>

#include "Force.h"
#include "Vec3.h"
#include "internal/windowsExport.h"

namespace OpenMM {
class OPENMM_EXPORT System {
public:
    System();
    ~System();
    int getNumParticles() const { return (int)masses.size(); }
    int addParticle(double mass) { masses.push_back(mass); return (int)masses.size() - 1; }
    double getParticleMass(int index) const;
    int addForce(Force* force) { forces.push_back(force); return (int)forces.size() - 1; }
    int getNumForces() const { return (int)forces.size(); }
    Force& getForce(int index);
    const Force& getForce(int index) const;
    void getDefaultPeriodicBoxVectors(Vec3& a, Vec3& b, Vec3& c) const;
    void setDefaultPeriodicBoxVectors(const Vec3& a, const Vec3& b, const Vec3& c);
    bool usesPeriodicBoundaryConditions() const;

private:
    Vec3 periodicBoxVectors[3];
    std::vector<double> masses;
    std::vector<Force*> forces;
};
}  // namespace OpenMM
#endif
