// Library-level C ABI entry points (version / target). Kernel entry points live with their kernels.
#include "common.hpp"

extern "C" {

int gtsfm_hip_abi_version(void) { return 101; }

const char* gtsfm_hip_target(void) { return "gfx950"; }

}  // extern "C"
