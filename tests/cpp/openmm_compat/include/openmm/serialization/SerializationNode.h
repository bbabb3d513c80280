// TEST INFRASTRUCTURE ONLY (openmm_compat): OpenMM::SerializationNode with OpenMM's
// signatures -- a named node with string properties (ints and doubles stored as text; doubles
// with 17 significant digits, which round-trip every fp64 value) and ordered children.
#ifndef OPENMM_SERIALIZATIONNODE_H_
#define OPENMM_SERIALIZATIONNODE_H_
#include <map>
#include <string>
#include <vector>

#include "../internal/windowsExport.h"

namespace OpenMM {
class OPENMM_EXPORT SerializationNode {
public:
    const std::string& getName() const { return name; }
    void setName(const std::string& n) { name = n; }
    const std::vector<SerializationNode>& getChildren() const { return children; }
    std::vector<SerializationNode>& getChildren() { return children; }
    const SerializationNode& getChildNode(const std::string& name) const;
    SerializationNode& getChildNode(const std::string& name);
    const std::map<std::string, std::string>& getProperties() const { return properties; }
    bool hasProperty(const std::string& name) const { return properties.count(name) != 0; }
    const std::string& getStringProperty(const std::string& name) const;
    const std::string& getStringProperty(const std::string& name, const std::string& defaultValue) const;
    SerializationNode& setStringProperty(const std::string& name, const std::string& value);
    int getIntProperty(const std::string& name) const;
    int getIntProperty(const std::string& name, int defaultValue) const;
    SerializationNode& setIntProperty(const std::string& name, int value);
    bool getBoolProperty(const std::string& name) const;
    bool getBoolProperty(const std::string& name, bool defaultValue) const;
    SerializationNode& setBoolProperty(const std::string& name, bool value);
    double getDoubleProperty(const std::string& name) const;
    double getDoubleProperty(const std::string& name, double defaultValue) const;
    SerializationNode& setDoubleProperty(const std::string& name, double value);
    SerializationNode& createChildNode(const std::string& name);

private:
    std::string name;
    std::vector<SerializationNode> children;
    std::map<std::string, std::string> properties;
};
}  // namespace OpenMM
#endif
