// TEST INFRASTRUCTURE ONLY (openmm_compat): CoulForce.h includes this header; nothing in the
// plugin uses OpenMM::Context itself.
#ifndef OPENMM_CONTEXT_H_
#define OPENMM_CONTEXT_H_
#include "internal/windowsExport.h"
namespace OpenMM {
class Context;
}
#endif
