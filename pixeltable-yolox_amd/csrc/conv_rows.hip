// conv_rows dispatch: geometry check + dtype switch; kernels in conv_rows.hpp,
// instantiated per dtype in conv_rows_{bf16,f16,f32}.hip.
#include "conv_common.hpp"

namespace yxh {

template <typename T>
int conv_rows_dispatch_t(int id, const ConvParams& p, int ks, hipStream_t st);
extern template int conv_rows_dispatch_t<bf16>(int, const ConvParams&, int, hipStream_t);
extern template int conv_rows_dispatch_t<f16>(int, const ConvParams&, int, hipStream_t);
extern template int conv_rows_dispatch_t<float>(int, const ConvParams&, int, hipStream_t);

int conv_rows_dispatch(int dtype, int id, const ConvParams& p, int ks, hipStream_t st) {
    if (p.taps != 9 || p.kw != 3 || p.pad != 1 || (p.stride != 1 && p.stride != 2) || p.nsrc != 1 || p.sup[0]) {
        set_error("conv_rows needs a single-source 3x3 pad-1 conv with stride 1 or 2");
        return YXH_EUNSUPPORTED;
    }
    if (dtype == YXH_BF16) return conv_rows_dispatch_t<bf16>(id, p, ks, st);
    if (dtype == YXH_F16) return conv_rows_dispatch_t<f16>(id, p, ks, st);
    return conv_rows_dispatch_t<float>(id, p, ks, st);
}

}  // namespace yxh
