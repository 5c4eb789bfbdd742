// Store-path probe (diagnostic, not part of the library): how fast can a grid
// shaped like the eye pass write a 3840x2160 RGBA f32 frame, as a function of
// pixels per lane and workgroup size?  hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int W = 3840, H = 2160;

template <int PPL>  // pixels per lane, consecutive columns
__global__ void store_rgba(float4* __restrict__ out, float v) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int waves = blockDim.x >> 6;
    const int xb = blockIdx.x * 64 * PPL;
    const int y = blockIdx.y * waves + wave;
    if (y >= H) return;
#pragma unroll
    for (int p = 0; p < PPL; ++p) {
        const int x = xb + p * 64 + lane;  // each store instruction: 64 consecutive pixels
        if (x < W) out[(size_t)y * W + x] = make_float4(v + x, v, v + y, 1.0f);
    }
}

template <int PPL>
__global__ void store_f64(double* __restrict__ out, double v) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int waves = blockDim.x >> 6;
    const int xb = blockIdx.x * 64 * PPL;
    const int y = blockIdx.y * waves + wave;
    if (y >= H) return;
#pragma unroll
    for (int p = 0; p < PPL; ++p) {
        const int x = xb + p * 64 + lane;
        if (x < W) out[(size_t)y * W + x] = v + x;
    }
}

__global__ void empty_kernel(float* out, int flag) {
    if (flag == 12345) out[threadIdx.x] = 0.0f;
}

// a kernel that needs many VGPRs (live f64 values) but does no memory work
__global__ void heavy_regs_kernel(float* out, int flag, double seed) {
    double v[40];
#pragma unroll
    for (int i = 0; i < 40; ++i) v[i] = seed * (threadIdx.x + i);
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < 40; ++i) acc += v[i] * v[(i + 7) % 40];
    if (flag == 12345 || acc == -1.0) out[threadIdx.x] = (float)acc;
}

template <typename F>
static float time_it(F f, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 5; ++i) f();
    hipEventRecord(a);
    for (int i = 0; i < iters; ++i) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1000.0f / iters;  // us
}

int main() {
    float4* o4;
    double* o8;
    if (hipMalloc(&o4, sizeof(float4) * W * H) != hipSuccess || hipMalloc(&o8, sizeof(double) * W * H) != hipSuccess)
        return 1;
    const double mb4 = 16.0 * W * H / 1e6, mb8 = 8.0 * W * H / 1e6;
#define RGBA(P, B)                                                                                            \
    {                                                                                                          \
        dim3 g((W + 64 * P - 1) / (64 * P), (H + (B / 64) - 1) / (B / 64));                                    \
        float us = time_it([&] { hipLaunchKernelGGL(store_rgba<P>, g, dim3(B), 0, 0, o4, 1.0f); }, 50);        \
        printf("rgba  ppl=%d block=%4d waves=%7u  %7.2f us  %6.2f TB/s\n", P, B, g.x * g.y * (B / 64), us,   \
               mb4 / us / 1e6 * 1e6 / 1e6);                                                                    \
    }
#define F64(P, B)                                                                                             \
    {                                                                                                          \
        dim3 g((W + 64 * P - 1) / (64 * P), (H + (B / 64) - 1) / (B / 64));                                    \
        float us = time_it([&] { hipLaunchKernelGGL(store_f64<P>, g, dim3(B), 0, 0, o8, 1.0); }, 50);          \
        printf("f64   ppl=%d block=%4d waves=%7u  %7.2f us  %6.2f TB/s\n", P, B, g.x * g.y * (B / 64), us,   \
               mb8 / us / 1e6 * 1e6 / 1e6);                                                                    \
    }
    for (int wgs : {4050, 32400, 129600}) {
        float us = time_it([&] { hipLaunchKernelGGL(empty_kernel, dim3(wgs), dim3(256), 0, 0, (float*)o4, 0); }, 50);
        float us1 = time_it([&] { hipLaunchKernelGGL(empty_kernel, dim3(wgs), dim3(256), 1040, 0, (float*)o4, 0); }, 50);
        float us2 = time_it([&] { hipLaunchKernelGGL(heavy_regs_kernel, dim3(wgs), dim3(256), 0, 0, (float*)o4, 0, 1.0); }, 50);
        printf("empty kernel %6d WGs x 256: %6.2f us (with 1 KB dyn LDS %6.2f us; ~90-VGPR kernel %6.2f us)\n", wgs, us, us1, us2);
    }
    RGBA(1, 256) RGBA(2, 256) RGBA(4, 256) RGBA(8, 256) RGBA(1, 512) RGBA(1, 1024) RGBA(4, 1024)
    F64(1, 256) F64(2, 256) F64(4, 256) F64(8, 256) F64(4, 1024)
    hipFree(o4);
    hipFree(o8);
    return 0;
}
