// ISA probe: one instantiation of k_rows_pl alone, so its VGPR / spill /
// waitcnt shape can be read in seconds:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --offload-device-only -S \
//         -I include [-DKWP=5 -DNTP=1024 -DNKP=1 -DWKP=3 -DVP=0] -o /tmp/probe.s tools/isa/probe_rows_pl.hip
#include "../../parfastaai_amd/csrc/pfaai_rows_pl.hpp"
#ifndef KWP
#define KWP 5
#endif
#ifndef NTP
#define NTP 1024
#endif
#ifndef NKP
#define NKP 1
#endif
#ifndef WKP
#define WKP 3
#endif
#ifndef MODEP
#define MODEP 0
#endif
#ifndef BIGFP
#define BIGFP false
#endif
#ifndef VP
#define VP 0
#endif

template __global__ void pfaai::k_rows_pl<MODEP, KWP, NTP, 8, false, NKP, BIGFP, WKP, VP>(
    pfaai::Dev, int64_t, int32_t, int32_t, uint32_t, const unsigned long long*, double*, double*, int32_t*,
    unsigned long long*, unsigned long long*);
