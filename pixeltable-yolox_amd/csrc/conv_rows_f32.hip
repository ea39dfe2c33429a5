// conv_rows variants for float (see conv_rows.hpp)
#include "conv_rows.hpp"

namespace yxh {
template int conv_rows_dispatch_t<float>(int id, const ConvParams& p, int ks, hipStream_t st);
}  // namespace yxh
