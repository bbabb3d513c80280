// TEST INFRASTRUCTURE ONLY (openmm_compat): OpenMM::OpenMMException with OpenMM's signatures.
#ifndef OPENMM_OPENMMEXCEPTION_H_
#define OPENMM_OPENMMEXCEPTION_H_
#include <exception>
#include <string>

#include "internal/windowsExport.h"

namespace OpenMM {
class OPENMM_EXPORT OpenMMException : public std::exception {
public:
    explicit OpenMMException(const std::string& message) : message(message) {}
    ~OpenMMException() throw() {}
    const char* what() const throw() { return message.c_str(); }

private:
    std::string message;
};
}  // namespace OpenMM
#endif
