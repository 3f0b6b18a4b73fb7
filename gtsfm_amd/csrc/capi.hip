// Library-level C ABI entry points (version / target). Kernel entry points live with their kernels.
#include "common.hpp"

extern "C" {

// 2.00: gtsfm_ransac_E_batched gained d_n_models; gtsfm_compact_verified added
// 3.01: gtsfm_ba2_batched gained the relative-pose prior inputs d_prior_Rt / d_prior_sigmas
// 4.00: gtsfm_superpoint_batched gained d_masks (SuperPoint image masks); gtsfm_ransac_E_batched / _F_batched
//       reject more argument shapes with GTSFM_ERR_ARG
// 4.01: gtsfm_netvlad_* added (NetVLAD global descriptor)
// 4.02: gtsfm_match_rerank_stats added (F16_RERANK certificate counts)
int gtsfm_hip_abi_version(void) { return GTSFM_HIP_ABI_VERSION; }

const char* gtsfm_hip_target(void) { return "gfx950"; }

}  // extern "C"
