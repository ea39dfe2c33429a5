// conv_rows variants for bf16 (see conv_rows.hpp)
#include "conv_rows.hpp"

namespace yxh {
template int conv_rows_dispatch_t<bf16>(int id, const ConvParams& p, int ks, hipStream_t st);
}  // namespace yxh
