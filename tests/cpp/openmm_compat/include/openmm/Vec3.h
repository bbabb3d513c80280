// TEST INFRASTRUCTURE ONLY (openmm_compat): OpenMM::Vec3 (three packed doubles, the layout
// the plugin relies on when it passes vector<Vec3> storage across the C-ABI).
#ifndef OPENMM_VEC3_H_
#define OPENMM_VEC3_H_
#include <cassert>

namespace OpenMM {
class Vec3 {
public:
    Vec3() { data[0] = data[1] = data[2] = 0.0; }
    Vec3(double x, double y, double z) { data[0] = x; data[1] = y; data[2] = z; }
    double operator[](int index) const { return data[index]; }
    double& operator[](int index) { return data[index]; }
    bool operator==(const Vec3& r) const { return data[0] == r[0] && data[1] == r[1] && data[2] == r[2]; }

private:
    double data[3];
};
}  // namespace OpenMM
#endif
