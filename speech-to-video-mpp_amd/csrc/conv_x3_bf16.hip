// bf16 instances of the split-fp32 implicit-GEMM convolution (S2V_PREC_BF16X3; conv_x3_impl.hpp).
#include "conv_x3_impl.hpp"

namespace s2v {
extern template bool launch_conv_x3_part<0, 1>(int, const ConvArgs &, int, bool, dim3, hipStream_t);
extern template bool launch_conv_x3_part<0, 2>(int, const ConvArgs &, int, bool, dim3, hipStream_t);
template bool launch_conv_x3_part<0, 0>(int, const ConvArgs &, int, bool, dim3, hipStream_t);
template int launch_conv_x3<0>(int cfg, const ConvArgs &a, int amode, bool bkn, dim3 grid, hipStream_t s);
template int launch_conv_x3_group<0>(int cfg, const ConvGroup &g, dim3 grid, hipStream_t s);
}  // namespace s2v
