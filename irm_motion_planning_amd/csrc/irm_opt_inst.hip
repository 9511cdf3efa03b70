// irm_opt_inst.hip — one instantiation unit of the optimiser templates, compiled once per
// shape by irm_motion_planning_amd/build.py (in parallel):
//   -DIRM_INST_DYN=<D>                           k_optimize<DynShape<D>> + k_forward<D>
//   -DIRM_INST_FIX_D=<D> -DIRM_INST_FIX_N=<N>      dispatch + lean k_gd_single<FixShape<D, N, 32>>
//   -DIRM_INST_GEN_D=<D> -DIRM_INST_GEN_N=<N>      general k_optimize<FixShape<D, N, 32>>
//   -DIRM_INST_DENSE_D=<D> -DIRM_INST_DENSE_N=<N>  k_lean<DenseShape<D, N>> (the dense operator's GD loop)
// (the general kernels get their own unit so that build.py can pick their machine scheduler)
#include "irm_kernels_impl.hpp"

namespace irm {
#if defined(IRM_INST_DYN)
template hipError_t launch_general_shape<DynShape<IRM_INST_DYN>>(const KParams&, hipStream_t, LaunchDesc*);
template hipError_t launch_optimize_shape<DynShape<IRM_INST_DYN>>(const KParams&, hipStream_t, LaunchDesc*);
template hipError_t launch_forward_dim<IRM_INST_DYN>(const KParams&, int, hipStream_t);
#elif defined(IRM_INST_FIX_D) && defined(IRM_INST_FIX_N)
extern template hipError_t launch_general_shape<FixShape<IRM_INST_FIX_D, IRM_INST_FIX_N, 32>>(const KParams&,
                                                                                               hipStream_t, LaunchDesc*);
template hipError_t launch_optimize_shape<FixShape<IRM_INST_FIX_D, IRM_INST_FIX_N, 32>>(const KParams&, hipStream_t,
                                                                                        LaunchDesc*);
#elif defined(IRM_INST_DENSE_D) && defined(IRM_INST_DENSE_N)
template hipError_t launch_dense_shape<DenseShape<IRM_INST_DENSE_D, IRM_INST_DENSE_N>>(const KParams&, hipStream_t,
                                                                                      LaunchDesc*, bool*);
#elif defined(IRM_INST_GEN_D) && defined(IRM_INST_GEN_N)
template hipError_t launch_general_shape<FixShape<IRM_INST_GEN_D, IRM_INST_GEN_N, 32>>(const KParams&, hipStream_t,
                                                                                       LaunchDesc*);
#else
#error "irm_opt_inst.hip needs IRM_INST_DYN, IRM_INST_FIX_D/N, IRM_INST_DENSE_D/N or IRM_INST_GEN_D/N"
#endif
}  // namespace irm
