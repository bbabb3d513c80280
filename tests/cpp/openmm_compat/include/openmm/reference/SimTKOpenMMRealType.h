// TEST INFRASTRUCTURE ONLY (openmm_compat): OpenMM's physical constants header, reduced to the
// Coulomb constant the reference reads (ReferenceCoulKernels.cpp:7).  Its value differs between
// OpenMM versions: 138.935456 (7.x) and 138.93545764438198 (8.x, CODATA 2018); the compat build
// compiles the plugin once per value (-DCOMPAT_ONE_4PI_EPS0=...) to show that the plugin takes
// whatever the OpenMM it is built against defines.
#ifndef OPENMM_SIMTKOPENMMREALTYPE_H_
#define OPENMM_SIMTKOPENMMREALTYPE_H_
#ifndef COMPAT_ONE_4PI_EPS0
#define COMPAT_ONE_4PI_EPS0 138.935456
#endif
#define ONE_4PI_EPS0 COMPAT_ONE_4PI_EPS0
#endif
