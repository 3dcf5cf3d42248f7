// ISA probe: one instantiation of k_rows_pl alone, so its VGPR / spill /
// waitcnt shape can be read in seconds:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --offload-device-only -S \
//         -I include [-DNKP=1 -DS5FP=true -DBRP=true] -o /tmp/probe.s tools/isa/probe_rows_pl.hip
#include "../../parfastaai_amd/csrc/pfaai_rows_pl.hpp"
#ifndef NKP
#define NKP 1
#endif
#ifndef S5FP
#define S5FP true
#endif
#ifndef VARP
#define VARP 0
#endif
#ifndef WKP
#define WKP 3
#endif
#ifndef BRP
#define BRP true
#endif

template __global__ void pfaai::k_rows_pl<0, 5, 1024, 8, false, NKP, false, S5FP, BRP, VARP, WKP>(
    pfaai::Dev, int64_t, int32_t, int32_t, uint32_t, const unsigned long long*, double*, double*, int32_t*,
    unsigned long long*, unsigned long long*);
