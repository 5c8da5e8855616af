// devknobs.hpp — development A/B knobs.  The environment is
// read only in a -DDDLO_DEV build (`make dev`); the default library ignores
// it, and its behaviour is set through the C-ABI alone (gicp_set_option,
// gicp_set_default_option, the params structs).
#pragma once
#include <cstdlib>

namespace ddlo {

inline const char* dev_getenv(const char* name) {
#ifdef DDLO_DEV
  return std::getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

}  // namespace ddlo
