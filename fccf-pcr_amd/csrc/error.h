// error.h — the exception the library's internals throw; the C-ABI entry points turn
// it into its FCCF_E_* status code (no exception crosses the ABI).
#pragma once
#include <stdexcept>
#include <string>

namespace fccf {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

}  // namespace fccf
