// irm_opt_inst.hip — one instantiation unit of the optimiser templates, compiled once per
// shape by irm_motion_planning_amd/build.py (in parallel):
//   -DIRM_INST_DYN=<D>                       k_optimize<DynShape<D>> + k_forward<D>
//   -DIRM_INST_FIX_D=<D> -DIRM_INST_FIX_N=<N>  k_optimize<FixShape<D, N, 32>>
#include "irm_kernels_impl.hpp"

namespace irm {
#if defined(IRM_INST_DYN)
template hipError_t launch_optimize_shape<DynShape<IRM_INST_DYN>>(const KParams&, hipStream_t);
template hipError_t launch_forward_dim<IRM_INST_DYN>(const KParams&, int, hipStream_t);
#elif defined(IRM_INST_FIX_D) && defined(IRM_INST_FIX_N)
template hipError_t launch_optimize_shape<FixShape<IRM_INST_FIX_D, IRM_INST_FIX_N, 32>>(const KParams&, hipStream_t);
#else
#error "irm_opt_inst.hip needs IRM_INST_DYN or IRM_INST_FIX_D/IRM_INST_FIX_N"
#endif
}  // namespace irm
