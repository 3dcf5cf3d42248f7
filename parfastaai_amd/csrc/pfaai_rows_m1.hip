// pfaai_rows_m1.hip -- the row kernels of mode 1 (query subset),
// instantiated in a translation unit of their own so the modes compile in
// parallel (tools/build_native.py).
#include "pfaai_launch.hpp"

namespace pfaai_impl {
template void launch_rows<1>(pfaai_ctx* c, int64_t rb, int64_t re, uint32_t flags, double* aji, double* S,
                             int32_t* N, hipStream_t s);
template void preload_rows<1>();
}  // namespace pfaai_impl
