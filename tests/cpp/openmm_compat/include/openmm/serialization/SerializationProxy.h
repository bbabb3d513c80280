// TEST INFRASTRUCTURE ONLY (openmm_compat): OpenMM::SerializationProxy -- the per-class
// serializer that OpenMM's XmlSerializer looks up by C++ type (serialize) or by the document's
// "type" property (deserialize).
#ifndef OPENMM_SERIALIZATIONPROXY_H_
#define OPENMM_SERIALIZATIONPROXY_H_
#include <string>
#include <typeinfo>

#include "../internal/windowsExport.h"
#include "SerializationNode.h"

namespace OpenMM {
class OPENMM_EXPORT SerializationProxy {
public:
    SerializationProxy(const std::string& typeName) : typeName(typeName) {}
    virtual ~SerializationProxy() {}
    const std::string& getTypeName() const { return typeName; }
    virtual void serialize(const void* object, SerializationNode& node) const = 0;
    virtual void* deserialize(const SerializationNode& node) const = 0;
    static void registerProxy(const std::type_info& type, const SerializationProxy* proxy);
    static const SerializationProxy& getProxy(const std::string& typeName);
    static const SerializationProxy& getProxy(const std::type_info& type);

private:
    std::string typeName;
};
}  // namespace OpenMM
#endif
