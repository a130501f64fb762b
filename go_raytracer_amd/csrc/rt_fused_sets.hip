// rt_fused_sets.hip — fused-kernel instantiations compiled with their own code-generation
// flags (Makefile: LLVM's iterative-ILP machine scheduler); the list and the measurement
// are in rt_fused.h (RT_FUSED_ILP_KERNELS).  Everything else is in rt_render.hip.
#include <hip/hip_runtime.h>

#include "rt_internal.h"
#include "rt_fused.h"

namespace rt {
#define RT_FUSED_INST(L, F, T) template __global__ void k_fused<L, F, T>(Params);
RT_FUSED_ILP_KERNELS(RT_FUSED_INST)
#undef RT_FUSED_INST
}  // namespace rt
