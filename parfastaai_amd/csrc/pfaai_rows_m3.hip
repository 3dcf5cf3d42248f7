// pfaai_rows_m3.hip -- the row kernels of the full-row mode (kModeFull: the
// dense output rows of pfaai_stream_matrix), in a translation unit of their
// own so the modes compile in parallel (tools/build_native.py).
#include "pfaai_launch.hpp"

namespace pfaai_impl {
template void launch_rows<kModeFull>(pfaai_ctx* c, int64_t rb, int64_t re, uint32_t flags, double* aji, double* S,
                                     int32_t* N, hipStream_t s);
template void preload_rows<3>();
}  // namespace pfaai_impl
