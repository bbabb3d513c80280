// TEST INFRASTRUCTURE ONLY — a C++ class with the public API of CoulPlugin::CoulForce
// (reference: openmmapi/include/CoulForce.h:22-133; same names, argument types and order,
// defaults cutoff 1.0 nm, Ewald tolerance 1e-4, no PBC, CoulForce.cpp:12-16) but without the
// OpenMM::Force base, which this image cannot provide.  It lets the plugin's force adapter
// (openmm-chargeflux_amd/plugin/include/CoulHipMarshal.h, a template over the force type) be
// compiled and exercised here; with OpenMM the adapter is instantiated on the real CoulForce.
// Storage is this file's own (per-term structs), not the reference's flat vectors.
#ifndef COUL_FORCE_STAND_IN_H_
#define COUL_FORCE_STAND_IN_H_

#include <stdexcept>
#include <vector>

namespace CoulPlugin {

class CoulForce {
public:
    CoulForce() = default;

    void addParticle(double charge, double sigma, double epsilon) { particles_.push_back({charge, sigma, epsilon}); }
    int getNumParticles() const { return (int)particles_.size(); }
    void getParticleParameters(int index, double& charge, double& sigma, double& epsilon) const {
        const Particle& p = at(particles_, index);
        charge = p.q; sigma = p.sig; epsilon = p.eps;
    }
    void setParticleParameters(int index, double charge, double sigma, double epsilon) {
        at(particles_, index) = {charge, sigma, epsilon};
    }

    double getCutoffDistance() const { return cutoff_; }
    void setCutoffDistance(double cutoff) { cutoff_ = cutoff; }
    bool usesPeriodicBoundaryConditions() const { return pbc_; }
    void setUsesPeriodicBoundaryConditions(bool ifPeriod) { pbc_ = ifPeriod; }

    void addException(int p1, int p2) { exceptions_.push_back({p1, p2}); }
    int getNumExceptions() const { return (int)exceptions_.size(); }
    void getExceptionParameters(const int index, int& p1, int& p2) const {
        const Pair& e = at(exceptions_, index);
        p1 = e.a; p2 = e.b;
    }

    void setEwaldErrorTolerance(double tol) { tol_ = tol; }
    double getEwaldErrorTolerance() const { return tol_; }

    void addFluxBond(int p1, int p2, double k, double b) { bonds_.push_back({p1, p2, k, b}); }
    void getFluxBondParameters(int index, int& p1, int& p2, double& k, double& b) const {
        const Bond& t = at(bonds_, index);
        p1 = t.p1; p2 = t.p2; k = t.k; b = t.b;
    }
    int getNumFluxBonds() const { return (int)bonds_.size(); }

    void addFluxAngle(int p1, int p2, int p3, double k, double theta) { angles_.push_back({p1, p2, p3, k, theta}); }
    void getFluxAngleParameters(int index, int& p1, int& p2, int& p3, double& k, double& theta) const {
        const Angle& t = at(angles_, index);
        p1 = t.p1; p2 = t.p2; p3 = t.p3; k = t.k; theta = t.theta;
    }
    int getNumFluxAngles() const { return (int)angles_.size(); }

    void addFluxWater(int po, int ph1, int ph2, double k1, double k2, double kub, double b0, double ub0) {
        waters_.push_back({po, ph1, ph2, k1, k2, kub, b0, ub0});
    }
    void getFluxWaterParameters(int index, int& po, int& ph1, int& ph2, double& k1, double& k2, double& kub,
                                double& b0, double& ub0) const {
        const Water& w = at(waters_, index);
        po = w.o; ph1 = w.h1; ph2 = w.h2; k1 = w.k1; k2 = w.k2; kub = w.kub; b0 = w.b0; ub0 = w.ub0;
    }
    int getNumFluxWaters() const { return (int)waters_.size(); }

private:
    struct Particle { double q, sig, eps; };
    struct Pair { int a, b; };
    struct Bond { int p1, p2; double k, b; };
    struct Angle { int p1, p2, p3; double k, theta; };
    struct Water { int o, h1, h2; double k1, k2, kub, b0, ub0; };
    template <class T>
    static T& at(std::vector<T>& v, int i) {
        if (i < 0 || i >= (int)v.size()) throw std::out_of_range("CoulForce index out of range");
        return v[i];
    }
    template <class T>
    static const T& at(const std::vector<T>& v, int i) {
        if (i < 0 || i >= (int)v.size()) throw std::out_of_range("CoulForce index out of range");
        return v[i];
    }
    std::vector<Particle> particles_;
    std::vector<Pair> exceptions_;
    std::vector<Bond> bonds_;
    std::vector<Angle> angles_;
    std::vector<Water> waters_;
    double cutoff_ = 1.0;
    double tol_ = 1e-4;
    bool pbc_ = false;
};

}  // namespace CoulPlugin

#endif  // COUL_FORCE_STAND_IN_H_
