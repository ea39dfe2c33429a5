// conv_rows variants for f16 (see conv_rows.hpp)
#include "conv_rows.hpp"

namespace yxh {
template int conv_rows_dispatch_t<f16>(int id, const ConvParams& p, int ks, hipStream_t st);
}  // namespace yxh
