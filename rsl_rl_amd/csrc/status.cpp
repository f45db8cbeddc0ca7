// Version and status-code strings of the C ABI (include/rslrl_amd.h).
#include "../../include/rslrl_amd.h"

extern "C" int rslrl_abi_version(void) { return RSLRL_ABI_VERSION; }

extern "C" const char* rslrl_status_string(int status) {
    switch (status) {
        case RSLRL_OK: return "ok";
        case RSLRL_E_INVALID_ARGUMENT: return "invalid argument";
        case RSLRL_E_WORKSPACE_TOO_SMALL: return "workspace too small";
        case RSLRL_E_UNSUPPORTED: return "unsupported configuration";
        case RSLRL_E_MISALIGNED: return "misaligned pointer";
        case RSLRL_E_BAD_GENERATOR_STATE: return "bad torch CPU generator state blob";
        default: return status > 0 ? "HIP runtime error (status is a hipError_t)" : "unknown status";
    }
}
