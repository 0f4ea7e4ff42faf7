// f16 instances of the split-fp32 convolution, tile configurations of part 2 (conv_x3_impl.hpp
// launch_conv_x3_part; a translation unit of its own so the parts compile in parallel).
#include "conv_x3_impl.hpp"

namespace s2v {
template bool launch_conv_x3_part<1, 2>(int, const ConvArgs &, int, bool, dim3, hipStream_t);
}  // namespace s2v
