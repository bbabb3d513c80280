// TEST INFRASTRUCTURE ONLY (openmm_compat, see ../../README.md): OpenMM's export macro.
#ifndef OPENMM_WINDOWSEXPORT_H_
#define OPENMM_WINDOWSEXPORT_H_
#define OPENMM_EXPORT __attribute__((visibility("default")))
#endif
