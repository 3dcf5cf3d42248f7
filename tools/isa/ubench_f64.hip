// ubench_f64.hip -- issue cost of the fp64 / conversion / LDS instructions
// k_rows_pl's S5 is made of, measured on the whole chip at 8 waves per SIMD
// (the row kernel's occupancy).  Each thread runs U independent chains of one
// operation; the time per wave-instruction per SIMD is
//   t_kernel * clock * n_SIMDs / (waves * iters * U)
// with the clock taken from the run itself (s_memtime ticks over the kernel
// in wave 0 of workgroup 0).  Diagnostic tool, not product code:
//   hipcc --offload-arch=gfx950 -O3 -o tools/_build/ubench_f64 tools/isa/ubench_f64.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int U = 8;
constexpr int NT = 256;

__device__ __forceinline__ double exact_div_small(double c, double dd) {
    double y = __builtin_amdgcn_rcp(dd);
    const double e = __builtin_fma(-dd, y, 1.0);
    y = __builtin_fma(y, e, y);
    const double q = c * y;
    const double r = __builtin_fma(-dd, q, c);
    return __builtin_fma(r, y, q);
}

// OP: 0 fma_f64, 1 mul_f64, 2 rcp_f64, 3 cvt_f64_u32, 4 add_u32, 5 fma_f32,
//     6 S += exact_div_small(c, d) (ints in, cvt included),
//     7 S += table division (LDS 1/d, ds_read_b64, q = c*r, residual, fma),
//     8 rcp_f32, 9 ds_read_b64 at random-ish addresses (+ an add)
template <int OP>
__global__ __launch_bounds__(NT) void k_op(double* out, int iters, unsigned long long* ticks, int dmax) {
    __shared__ double rtab[2048];
    for (int i = threadIdx.x; i < 2048; i += NT) rtab[i] = 1.0 / (double)(i ? i : 1);
    __syncthreads();
    const unsigned long long t0 = __builtin_readcyclecounter();
    double a[U];
    float f[U];
    uint32_t u[U];
    const int tid = threadIdx.x + blockIdx.x * NT;
#pragma unroll
    for (int j = 0; j < U; ++j) {
        a[j] = 1.0 + 1e-3 * (tid + j);
        f[j] = 1.0f + 1e-3f * (tid + j);
        u[j] = tid * 7 + j;
    }
    const double x = 0.999999, y = 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < U; ++j) {
            if constexpr (OP == 0) a[j] = __builtin_fma(a[j], x, y);
            if constexpr (OP == 1) a[j] = a[j] * x;
            if constexpr (OP == 2) a[j] = __builtin_amdgcn_rcp(a[j]);
            if constexpr (OP == 3) a[j] = (double)(u[j] + (uint32_t)it) ;
            if constexpr (OP == 4) u[j] = u[j] + (uint32_t)it;
            if constexpr (OP == 5) f[j] = __builtin_fmaf(f[j], 0.999f, 1e-7f);
            if constexpr (OP == 6 || OP == 7) {
                const uint32_t c = (u[j] + (uint32_t)it) & 255u;
                const uint32_t d = c + ((u[j] >> 3) & 511u) + 1u;
                if constexpr (OP == 6) {
                    a[j] += exact_div_small((double)c, (double)d);
                } else {
                    const double r = rtab[d];
                    const double dd = (double)d, cc = (double)c;
                    const double q = cc * r;
                    const double e = __builtin_fma(-dd, q, cc);
                    a[j] += __builtin_fma(e, r, q);
                }
            }
            if constexpr (OP == 8) f[j] = __builtin_amdgcn_rcpf(f[j]);
            if constexpr (OP == 9) a[j] += rtab[(u[j] + (uint32_t)it * 37u) & 2047u];
        }
    }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < U; ++j) s += a[j] + (double)f[j] + (double)u[j];
    out[tid] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) *ticks = __builtin_readcyclecounter() - t0;
}

// Exactness of the table division: q = RN(c * r), r = RN(1/d) (a correctly
// rounded reciprocal, as 1.0 / d gives), residual e = fma(-d, q, c), result
// fma(e, r, q) -- against IEEE c / d for every 0 <= c <= min(d, 65535),
// 1 <= d < dlim.  Counts mismatches.
__global__ void k_check_tab(int dlim, unsigned long long* bad) {
    const int d = blockIdx.x + 1;
    if (d >= dlim) return;
    const double dd = (double)d, r = 1.0 / dd;
    unsigned long long nb = 0;
    const int cmax = d < 65535 ? d : 65535;
    for (int c = threadIdx.x; c <= cmax; c += blockDim.x) {
        const double cc = (double)c, q = cc * r, e = __builtin_fma(-dd, q, cc), z = __builtin_fma(e, r, q);
        if (z != cc / dd) ++nb;
    }
    if (nb) atomicAdd(bad, nb);
}

template <int OP>
void run(const char* name, int blocks, int iters, double* out, unsigned long long* ticks, int nsimd) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(NT), 0, 0, out, iters, ticks, 2048);  // warm
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(NT), 0, 0, out, iters, ticks, 2048);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long tk = 0;
    (void)hipMemcpy(&tk, ticks, sizeof(tk), hipMemcpyDeviceToHost);
    const double waves = (double)blocks * NT / 64.0;
    const double ops = waves * iters * U;        // wave-level operations
    const double per_simd = ops / nsimd;
    // cycles per op per SIMD at the nominal 2.4 GHz, and ns per op per SIMD
    printf("%-28s %8.3f ms  %7.3f ns/op/SIMD  %6.2f cyc@2.4GHz  (wave0 ticks %llu)\n", name, ms,
           ms * 1e6 / per_simd, ms * 1e-3 * 2.4e9 / per_simd, tk);
}

int main(int argc, char** argv) {
    int dev = 0;
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, dev);
    const int cus = p.multiProcessorCount, nsimd = cus * 4;
    const int blocks = cus * 8;  // 8 workgroups of 4 waves per CU = 8 waves per SIMD
    const int iters = argc > 1 ? atoi(argv[1]) : 4096;
    printf("%s, %d CUs, clock %d kHz\n", p.gcnArchName, cus, p.clockRate);
    double* out;
    unsigned long long* ticks;
    (void)hipMalloc(&out, sizeof(double) * blocks * NT);
    (void)hipMalloc(&ticks, 8);
    run<4>("add_u32", blocks, iters, out, ticks, nsimd);
    run<5>("fma_f32", blocks, iters, out, ticks, nsimd);
    run<8>("rcp_f32", blocks, iters, out, ticks, nsimd);
    run<0>("fma_f64", blocks, iters, out, ticks, nsimd);
    run<1>("mul_f64", blocks, iters, out, ticks, nsimd);
    run<2>("rcp_f64", blocks, iters, out, ticks, nsimd);
    run<3>("cvt_f64_u32 (+add)", blocks, iters, out, ticks, nsimd);
    run<9>("ds_read_b64 (+add_f64)", blocks, iters, out, ticks, nsimd);
    run<6>("div rcp+newton (S += c/d)", blocks, iters, out, ticks, nsimd);
    run<7>("div LDS table (S += c/d)", blocks, iters, out, ticks, nsimd);
    (void)hipMemset(ticks, 0, 8);
    const int dlim = 1 << 17;
    hipLaunchKernelGGL(k_check_tab, dim3(dlim), dim3(1024), 0, 0, dlim, ticks);
    unsigned long long bad = ~0ull;
    (void)hipMemcpy(&bad, ticks, 8, hipMemcpyDeviceToHost);
    printf("table division vs IEEE '/', 1 <= d < %d, 0 <= c <= min(d, 65535): %llu mismatches\n", dlim, bad);
    return 0;
}
