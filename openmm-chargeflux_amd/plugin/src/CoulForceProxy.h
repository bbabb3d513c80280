// CoulForceProxy.h — XML serialization of CoulPlugin::CoulForce for OpenMM's XmlSerializer
// (the reference registers no proxy, so a System holding a CoulForce cannot be
// saved or reloaded).  Registered by registerKernelFactories (HipCoulKernelFactory.cpp).
#ifndef COUL_FORCE_PROXY_H_
#define COUL_FORCE_PROXY_H_

#include "openmm/serialization/SerializationProxy.h"

namespace CoulPlugin {

class CoulForceProxy : public OpenMM::SerializationProxy {
public:
    CoulForceProxy();
    void serialize(const void* object, OpenMM::SerializationNode& node) const override;
    void* deserialize(const OpenMM::SerializationNode& node) const override;
};

}  // namespace CoulPlugin

#endif  // COUL_FORCE_PROXY_H_
