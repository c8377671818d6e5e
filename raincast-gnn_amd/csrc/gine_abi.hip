// Library identity and status strings (no device code).
#include "gine_common.hpp"

extern "C" int gine_abi_version(void) { return GINE_ABI_VERSION; }

extern "C" const char* gine_status_string(int status) {
  switch (status) {
    case GINE_OK: return "ok";
    case GINE_ERR_INVALID: return "invalid argument (null pointer, negative size or bad flag)";
    case GINE_ERR_DIM: return "unsupported channel count";
    case GINE_ERR_WORKSPACE: return "workspace too small";
    case GINE_ERR_TOO_LARGE: return "num_nodes or num_edges >= 2^31";
    default: break;
  }
  if (status >= GINE_ERR_HIP_BASE) return hipGetErrorString((hipError_t)(status - GINE_ERR_HIP_BASE));
  return "unknown status";
}
