// TEST INFRASTRUCTURE ONLY — libOpenMM.so of the openmm_compat tree (see README.md there):
// definitions behind the compat headers, so that the OpenMM plugin sources
// (openmm-chargeflux_amd/plugin/src) link and load here exactly as they would against an
// OpenMM install.  It is not OpenMM: it implements only the registry, kernel handles, System,
// the Reference/CPU platform classes and the serialization machinery those sources touch.
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <istream>
#include <map>
#include <memory>
#include <ostream>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "openmm/Force.h"
#include "openmm/Kernel.h"
#include "openmm/KernelFactory.h"
#include "openmm/OpenMMException.h"
#include "openmm/Platform.h"
#include "openmm/System.h"
#include "openmm/reference/ReferencePlatform.h"
#include "openmm/serialization/SerializationNode.h"
#include "openmm/serialization/SerializationProxy.h"
#include "openmm/serialization/XmlSerializer.h"

using namespace OpenMM;

// ---- Force / System -------------------------------------------------------------------------
int Force::getForceGroup() const { return forceGroup; }
void Force::setForceGroup(int group) {
    if (group < 0 || group > 31) throw OpenMMException("Force group must be between 0 and 31");
    forceGroup = group;
}
const std::string& Force::getName() const { return name; }
void Force::setName(const std::string& n) { name = n; }

System::System() {
    periodicBoxVectors[0] = Vec3(2, 0, 0);
    periodicBoxVectors[1] = Vec3(0, 2, 0);
    periodicBoxVectors[2] = Vec3(0, 0, 2);
}
System::~System() {
    for (Force* f : forces) delete f;
}
double System::getParticleMass(int index) const {
    if (index < 0 || index >= (int)masses.size()) throw OpenMMException("Index out of range");
    return masses[index];
}
Force& System::getForce(int index) {
    if (index < 0 || index >= (int)forces.size()) throw OpenMMException("Index out of range");
    return *forces[index];
}
const Force& System::getForce(int index) const {
    if (index < 0 || index >= (int)forces.size()) throw OpenMMException("Index out of range");
    return *forces[index];
}
void System::getDefaultPeriodicBoxVectors(Vec3& a, Vec3& b, Vec3& c) const {
    a = periodicBoxVectors[0];
    b = periodicBoxVectors[1];
    c = periodicBoxVectors[2];
}
void System::setDefaultPeriodicBoxVectors(const Vec3& a, const Vec3& b, const Vec3& c) {
    periodicBoxVectors[0] = a;
    periodicBoxVectors[1] = b;
    periodicBoxVectors[2] = c;
}
bool System::usesPeriodicBoundaryConditions() const {
    for (Force* f : forces)
        if (f->usesPeriodicBoundaryConditions()) return true;
    return false;
}

// ---- kernels --------------------------------------------------------------------------------
KernelImpl::KernelImpl(std::string n, const Platform& p) : name(n), platform(&p), referenceCount(0) {}
std::string KernelImpl::getName() const { return name; }
const Platform& KernelImpl::getPlatform() { return *platform; }

Kernel::Kernel() : impl(nullptr) {}
Kernel::Kernel(KernelImpl* i) : impl(i) {
    if (impl) impl->referenceCount++;
}
Kernel::Kernel(const Kernel& copy) : impl(copy.impl) {
    if (impl) impl->referenceCount++;
}
Kernel::~Kernel() {
    if (impl && --impl->referenceCount == 0) delete impl;
}
Kernel& Kernel::operator=(const Kernel& copy) {
    if (copy.impl) copy.impl->referenceCount++;
    if (impl && --impl->referenceCount == 0) delete impl;
    impl = copy.impl;
    return *this;
}
std::string Kernel::getName() const {
    if (!impl) throw OpenMMException("Kernel has not been initialized");
    return impl->getName();
}
const KernelImpl& Kernel::getImpl() const { return *impl; }
KernelImpl& Kernel::getImpl() { return *impl; }

// ---- platforms ------------------------------------------------------------------------------
static std::vector<Platform*>& platforms() {
    static std::vector<Platform*> p;
    return p;
}

Platform::~Platform() {
    std::set<KernelFactory*> unique;
    for (auto& kv : kernelFactories) unique.insert(kv.second);
    for (KernelFactory* f : unique) delete f;
}
void Platform::registerKernelFactory(const std::string& name, KernelFactory* factory) {
    kernelFactories[name] = factory;   // as in OpenMM: a later registration replaces the earlier one
}
bool Platform::supportsKernels(const std::vector<std::string>& kernelNames) const {
    for (const std::string& n : kernelNames)
        if (kernelFactories.find(n) == kernelFactories.end()) return false;
    return true;
}
Kernel Platform::createKernel(const std::string& name, ContextImpl& context) const {
    auto it = kernelFactories.find(name);
    if (it == kernelFactories.end())
        throw OpenMMException("Called createKernel() on a Platform which does not support the requested kernel");
    return Kernel(it->second->createKernelImpl(name, *this, context));
}
void Platform::registerPlatform(Platform* platform) { platforms().push_back(platform); }
int Platform::getNumPlatforms() { return (int)platforms().size(); }
Platform& Platform::getPlatform(int index) {
    if (index < 0 || index >= getNumPlatforms()) throw OpenMMException("Invalid platform index");
    return *platforms()[index];
}
Platform& Platform::getPlatformByName(const std::string& name) {
    for (Platform* p : platforms())
        if (p->getName() == name) return *p;
    throw OpenMMException("There is no registered Platform called \"" + name + "\"");
}

ReferencePlatform::ReferencePlatform() {}

ReferencePlatform::PlatformData::PlatformData(const System& system)
    : numParticles(system.getNumParticles()), stepCount(0), time(0.0) {
    positions = new std::vector<Vec3>(numParticles);
    velocities = new std::vector<Vec3>(numParticles);
    forces = new std::vector<Vec3>(numParticles);
    periodicBoxSize = new Vec3();
    periodicBoxVectors = new Vec3[3];
}
ReferencePlatform::PlatformData::~PlatformData() {
    delete (std::vector<Vec3>*)positions;
    delete (std::vector<Vec3>*)velocities;
    delete (std::vector<Vec3>*)forces;
    delete (Vec3*)periodicBoxSize;
    delete[] (Vec3*)periodicBoxVectors;
}

namespace {
// OpenMM's CPU platform derives from ReferencePlatform (its contexts carry ReferencePlatform::
// PlatformData); a non-Reference platform stands for OpenCL / CUDA / HIP, where the plugin's
// host-buffer kernel must NOT attach.
class CompatCpuPlatform : public ReferencePlatform {
public:
    const std::string& getName() const {
        static const std::string name = "CPU";
        return name;
    }
};
class CompatDevicePlatform : public Platform {
public:
    const std::string& getName() const {
        static const std::string name = "OpenCL";
        return name;
    }
    double getSpeed() const { return 10; }
    bool supportsDoublePrecision() const { return true; }
};
}  // namespace

// what OpenMM's library constructor and platform plugins would register
extern "C" OPENMM_EXPORT void openmm_compat_register_platforms() {
    if (!platforms().empty()) return;
    Platform::registerPlatform(new ReferencePlatform());
    Platform::registerPlatform(new CompatCpuPlatform());
    Platform::registerPlatform(new CompatDevicePlatform());
}

// ---- serialization --------------------------------------------------------------------------
const SerializationNode& SerializationNode::getChildNode(const std::string& n) const {
    for (const SerializationNode& c : children)
        if (c.getName() == n) return c;
    throw OpenMMException("Unknown child '" + n + "' in node '" + name + "'");
}
SerializationNode& SerializationNode::getChildNode(const std::string& n) {
    for (SerializationNode& c : children)
        if (c.getName() == n) return c;
    throw OpenMMException("Unknown child '" + n + "' in node '" + name + "'");
}
const std::string& SerializationNode::getStringProperty(const std::string& n) const {
    auto it = properties.find(n);
    if (it == properties.end()) throw OpenMMException("Unknown property '" + n + "' in node '" + name + "'");
    return it->second;
}
const std::string& SerializationNode::getStringProperty(const std::string& n, const std::string& d) const {
    auto it = properties.find(n);
    return it == properties.end() ? d : it->second;
}
SerializationNode& SerializationNode::setStringProperty(const std::string& n, const std::string& v) {
    properties[n] = v;
    return *this;
}
int SerializationNode::getIntProperty(const std::string& n) const { return std::atoi(getStringProperty(n).c_str()); }
int SerializationNode::getIntProperty(const std::string& n, int d) const {
    return hasProperty(n) ? getIntProperty(n) : d;
}
SerializationNode& SerializationNode::setIntProperty(const std::string& n, int v) {
    return setStringProperty(n, std::to_string(v));
}
bool SerializationNode::getBoolProperty(const std::string& n) const {
    const std::string& v = getStringProperty(n);
    return v == "true" || v == "1";
}
bool SerializationNode::getBoolProperty(const std::string& n, bool d) const {
    return hasProperty(n) ? getBoolProperty(n) : d;
}
SerializationNode& SerializationNode::setBoolProperty(const std::string& n, bool v) {
    return setStringProperty(n, v ? "true" : "false");
}
double SerializationNode::getDoubleProperty(const std::string& n) const {
    return std::strtod(getStringProperty(n).c_str(), nullptr);
}
double SerializationNode::getDoubleProperty(const std::string& n, double d) const {
    return hasProperty(n) ? getDoubleProperty(n) : d;
}
SerializationNode& SerializationNode::setDoubleProperty(const std::string& n, double v) {
    char buf[40];
    std::snprintf(buf, sizeof(buf), "%.17g", v);
    return setStringProperty(n, buf);
}
SerializationNode& SerializationNode::createChildNode(const std::string& n) {
    children.emplace_back();
    children.back().setName(n);
    return children.back();
}

static std::map<std::string, const SerializationProxy*>& proxies_by_type() {
    static std::map<std::string, const SerializationProxy*> m;
    return m;
}
static std::map<std::string, const SerializationProxy*>& proxies_by_name() {
    static std::map<std::string, const SerializationProxy*> m;
    return m;
}
void SerializationProxy::registerProxy(const std::type_info& type, const SerializationProxy* proxy) {
    proxies_by_type()[type.name()] = proxy;
    proxies_by_name()[proxy->getTypeName()] = proxy;
}
const SerializationProxy& SerializationProxy::getProxy(const std::string& typeName) {
    auto it = proxies_by_name().find(typeName);
    if (it == proxies_by_name().end()) throw OpenMMException("There is no serialization proxy registered for type " + typeName);
    return *it->second;
}
const SerializationProxy& SerializationProxy::getProxy(const std::type_info& type) {
    auto it = proxies_by_type().find(type.name());
    if (it == proxies_by_type().end())
        throw OpenMMException(std::string("There is no serialization proxy registered for type ") + type.name());
    return *it->second;
}

namespace {
std::string xml_escape(const std::string& s) {
    std::string o;
    for (char c : s) {
        switch (c) {
            case '&': o += "&amp;"; break;
            case '<': o += "&lt;"; break;
            case '>': o += "&gt;"; break;
            case '"': o += "&quot;"; break;
            case '\'': o += "&apos;"; break;
            default: o += c;
        }
    }
    return o;
}
std::string xml_unescape(const std::string& s) {
    static const std::pair<const char*, char> ents[] = {{"&amp;", '&'}, {"&lt;", '<'}, {"&gt;", '>'},
                                                         {"&quot;", '"'}, {"&apos;", '\''}};
    std::string o;
    for (size_t i = 0; i < s.size();) {
        bool hit = false;
        if (s[i] == '&')
            for (const auto& e : ents) {
                const size_t n = std::string(e.first).size();
                if (s.compare(i, n, e.first) == 0) { o += e.second; i += n; hit = true; break; }
            }
        if (!hit) o += s[i++];
    }
    return o;
}
void write_node(const SerializationNode& node, const std::string& name, std::ostream& out, int depth) {
    const std::string pad(2 * depth, ' ');
    out << pad << '<' << name;
    for (const auto& kv : node.getProperties()) out << ' ' << kv.first << "=\"" << xml_escape(kv.second) << '"';
    if (node.getChildren().empty()) {
        out << "/>\n";
        return;
    }
    out << ">\n";
    for (const SerializationNode& c : node.getChildren()) write_node(c, c.getName(), out, depth + 1);
    out << pad << "</" << name << ">\n";
}

struct Parser {
    const std::string& s;
    size_t i = 0;
    explicit Parser(const std::string& text) : s(text) {}
    [[noreturn]] void fail(const std::string& what) {
        throw OpenMMException("XML parse error at offset " + std::to_string(i) + ": " + what);
    }
    void ws() {
        while (i < s.size() && std::isspace((unsigned char)s[i])) i++;
    }
    void skip_misc() {   // prolog, comments, whitespace
        for (;;) {
            ws();
            if (s.compare(i, 4, "<!--") == 0) {
                size_t e = s.find("-->", i);
                if (e == std::string::npos) fail("unterminated comment");
                i = e + 3;
            } else if (s.compare(i, 2, "<?") == 0) {
                size_t e = s.find("?>", i);
                if (e == std::string::npos) fail("unterminated declaration");
                i = e + 2;
            } else {
                return;
            }
        }
    }
    std::string name() {
        size_t b = i;
        while (i < s.size() && (std::isalnum((unsigned char)s[i]) || s[i] == '_' || s[i] == '-' || s[i] == '.' || s[i] == ':'))
            i++;
        if (b == i) fail("expected a name");
        return s.substr(b, i - b);
    }
    void element(SerializationNode& node) {
        skip_misc();
        if (i >= s.size() || s[i] != '<') fail("expected '<'");
        i++;
        node.setName(name());
        for (;;) {
            ws();
            if (s.compare(i, 2, "/>") == 0) { i += 2; return; }
            if (i < s.size() && s[i] == '>') { i++; break; }
            std::string key = name();
            ws();
            if (i >= s.size() || s[i] != '=') fail("expected '='");
            i++;
            ws();
            const char q = i < s.size() ? s[i] : 0;
            if (q != '"' && q != '\'') fail("expected a quoted value");
            size_t e = s.find(q, i + 1);
            if (e == std::string::npos) fail("unterminated value");
            node.setStringProperty(key, xml_unescape(s.substr(i + 1, e - i - 1)));
            i = e + 1;
        }
        for (;;) {
            skip_misc();
            if (s.compare(i, 2, "</") == 0) {
                i += 2;
                if (name() != node.getName()) fail("mismatched closing tag");
                ws();
                if (i >= s.size() || s[i] != '>') fail("expected '>'");
                i++;
                return;
            }
            element(node.createChildNode(""));
        }
    }
};
}  // namespace

void XmlSerializer::serialize(const SerializationNode* node, const std::string& rootName, std::ostream& stream) {
    stream << "<?xml version=\"1.0\" ?>\n";
    write_node(*node, rootName, stream, 0);
}

void* XmlSerializer::deserializeStream(std::istream& stream) {
    std::stringstream buf;
    buf << stream.rdbuf();
    const std::string text = buf.str();
    Parser p(text);
    SerializationNode root;
    p.element(root);
    const SerializationProxy& proxy = SerializationProxy::getProxy(root.getStringProperty("type"));
    return proxy.deserialize(root);
}

// compat only (not OpenMM API): the factory registered on `platform` for `name`, or null -- lets
// the test host call a plugin factory's createKernelImpl with a name OpenMM would never pass it
namespace OpenMM {
struct CompatRegistryAccess {
    static KernelFactory* get(const Platform& p, const std::string& name) {
        auto it = p.kernelFactories.find(name);
        return it == p.kernelFactories.end() ? nullptr : it->second;
    }
};
}  // namespace OpenMM
extern "C" OPENMM_EXPORT void* openmm_compat_factory(const char* platform, const char* name) {
    return CompatRegistryAccess::get(Platform::getPlatformByName(platform), name);
}
