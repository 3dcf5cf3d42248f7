// ISA probe: the benchmark instantiation of k_rows_v2 alone (see probe_rows_pl.hip)
#include "../../parfastaai_amd/csrc/pfaai_rows_v2.hpp"

template __global__ void pfaai::k_rows_v2<0, 5, false, false>(pfaai::Dev, int64_t, int32_t, int32_t, uint32_t,
                                                             const unsigned long long*, double*, double*, int32_t*,
                                                             unsigned long long*, unsigned long long*);
