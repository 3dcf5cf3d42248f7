// clkprobe.hip -- the shader clock the GPU is running at, measured from inside
// a kernel: one workgroup per CU spins on fp32 FMAs for a fixed wall time
// (wall_clock64(), the constant 100 MHz counter) and counts shader cycles over
// it (clock64()); cycles / wall seconds = the effective shader clock.  Used by
// tools/gpu/first_step.py to see whether the first runs after a load or an
// idle gap run at a lower clock (round 5).
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/gpu/libclkprobe.so tools/gpu/clkprobe.hip
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

__global__ __launch_bounds__(256) void k_clk(uint64_t wall_ticks, unsigned long long* out, float* sink) {
    const uint64_t w0 = wall_clock64();
    const uint64_t c0 = clock64();
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    uint64_t w = w0;
    while (w - w0 < wall_ticks) {
        for (int i = 0; i < 64; ++i) a = __builtin_fmaf(a, b, 1e-7f);
        w = wall_clock64();
    }
    const uint64_t c1 = clock64();
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = c1 - c0;
        out[2 * blockIdx.x + 1] = w - w0;
    }
    if (a == 12345.0f) sink[threadIdx.x] = a;  // keeps the loop
}

}  // namespace

extern "C" {

// the wall_clock64() rate of device `dev` in kHz (0 on error)
int clkprobe_wall_khz(int dev) {
    int khz = 0;
    return hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess ? khz : 0;
}

// Spin `us` microseconds (wall clock at wall_mhz) on `blocks` workgroups of `stream`; out (device,
// 2 * blocks u64): per block shader cycles and 100 MHz wall ticks.
int clkprobe_launch(void* stream, int blocks, int us, int wall_mhz, unsigned long long* out, float* sink) {
    if (blocks <= 0 || us <= 0 || !out || !sink) return 1;
    hipLaunchKernelGGL(k_clk, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream), (uint64_t)us * (uint64_t)wall_mhz, out,
                       sink);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // extern "C"
