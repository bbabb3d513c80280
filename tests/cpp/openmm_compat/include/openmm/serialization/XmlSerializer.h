// TEST INFRASTRUCTURE ONLY (openmm_compat): OpenMM::XmlSerializer -- the object's proxy fills a
// SerializationNode, the node is written as one XML element (properties as attributes, children
// as child elements) under rootName with a "type" attribute naming the proxy; deserialize
// parses the document and hands the root node to the proxy named by "type".
#ifndef OPENMM_XMLSERIALIZER_H_
#define OPENMM_XMLSERIALIZER_H_
#include <iosfwd>
#include <string>
#include <typeinfo>

#include "../internal/windowsExport.h"
#include "SerializationNode.h"
#include "SerializationProxy.h"

namespace OpenMM {
class OPENMM_EXPORT XmlSerializer {
public:
    template <class T>
    static void serialize(const T* object, const std::string& rootName, std::ostream& stream) {
        const SerializationProxy& proxy = SerializationProxy::getProxy(typeid(*object));
        SerializationNode node;
        proxy.serialize(object, node);
        node.setStringProperty("type", proxy.getTypeName());
        serialize(&node, rootName, stream);
    }
    template <class T>
    static T* deserialize(std::istream& stream) {
        return reinterpret_cast<T*>(deserializeStream(stream));
    }

private:
    static void serialize(const SerializationNode* node, const std::string& rootName, std::ostream& stream);
    static void* deserializeStream(std::istream& stream);
};
}  // namespace OpenMM
#endif
