// Store-pattern probe 2 (diagnostic, not part of the library): which way of
// writing a batch of RGBA f32 frames reaches the most HBM write bandwidth on
// MI355X?  Four 3840x2160 frames (531 MB) per launch, as the batched eye pass
// writes them.  hipcc --offload-arch=gfx950 -O3 store_probe2.hip -o store_probe2
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int W = 3840, H = 2160, NF = 4;
constexpr size_t NPX = (size_t)W * H * NF;

typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st(float4* p, float4 v, bool nt) {
    const f32x4 w = {v.x, v.y, v.z, v.w};
    if (nt) __builtin_nontemporal_store(w, reinterpret_cast<f32x4*>(p));
    else *reinterpret_cast<f32x4*>(p) = w;
}

// the eye pass's shape: 64x4 pixel tiles, one pixel per lane, grid z = frame
template <bool NT>
__global__ void tile64x4(float4* __restrict__ out) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x < W && y < H) st(out + (size_t)blockIdx.z * W * H + (size_t)y * W + x, make_float4(0.f, .2f, .2f, 1.f), NT);
}

// 256x1 tiles: a workgroup writes 4 KB contiguous
template <bool NT>
__global__ void tile256(float4* __restrict__ out) {
    const int x = blockIdx.x * 256 + threadIdx.x;
    const int y = blockIdx.y;
    if (x < W) st(out + (size_t)blockIdx.z * W * H + (size_t)y * W + x, make_float4(0.f, .2f, .2f, 1.f), NT);
}

// P consecutive pixels per lane (each lane 16*P contiguous bytes)
template <int P, bool NT>
__global__ void lane_run(float4* __restrict__ out) {
    const size_t i0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * P;
#pragma unroll
    for (int p = 0; p < P; ++p)
        if (i0 + p < NPX) st(out + i0 + p, make_float4(0.f, .2f, .2f, 1.f), NT);
}

// persistent grid-stride loop: G workgroups of 256 sweep the batch
template <bool NT>
__global__ void grid_stride(float4* __restrict__ out) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < NPX; i += stride)
        st(out + i, make_float4(0.f, .2f, .2f, 1.f), NT);
}

// a wave writes K consecutive 1 KB segments (K store instructions, 64*K pixels)
template <int K, bool NT>
__global__ void wave_span(float4* __restrict__ out) {
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const size_t base = wave * 64 * K;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const size_t i = base + (size_t)k * 64 + lane;
        if (i < NPX) st(out + i, make_float4(0.f, .2f, .2f, 1.f), NT);
    }
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
    return ms * 1000.0f / iters;
}

int main() {
    float4* o;
    if (hipMalloc(&o, sizeof(float4) * NPX) != hipSuccess) return 1;
    const double mb = 16.0 * NPX / 1e6;
    auto rep = [&](const char* name, float us) {
        printf("%-34s %8.2f us/launch  %6.2f us/frame  %5.2f TB/s\n", name, us, us / NF, mb / us);  // MB per us = TB/s
    };
    const int iters = 40;
    rep("tile64x4 cached", time_it([&] { hipLaunchKernelGGL(tile64x4<false>, dim3(W / 64, H / 4, NF), dim3(256), 0, 0, o); }, iters));
    rep("tile64x4 nontemporal", time_it([&] { hipLaunchKernelGGL(tile64x4<true>, dim3(W / 64, H / 4, NF), dim3(256), 0, 0, o); }, iters));
    rep("tile256 cached", time_it([&] { hipLaunchKernelGGL(tile256<false>, dim3(W / 256, H, NF), dim3(256), 0, 0, o); }, iters));
    rep("tile256 nontemporal", time_it([&] { hipLaunchKernelGGL(tile256<true>, dim3(W / 256, H, NF), dim3(256), 0, 0, o); }, iters));
#define RUN(P)                                                                                                   \
    rep("lane_run P=" #P " nt", time_it([&] { hipLaunchKernelGGL((lane_run<P, true>), dim3((unsigned)((NPX / P + 255) / 256)), dim3(256), 0, 0, o); }, iters)); \
    rep("lane_run P=" #P " cached", time_it([&] { hipLaunchKernelGGL((lane_run<P, false>), dim3((unsigned)((NPX / P + 255) / 256)), dim3(256), 0, 0, o); }, iters));
    RUN(2) RUN(4)
#define SPAN(K)                                                                                                  \
    rep("wave_span K=" #K " nt", time_it([&] { hipLaunchKernelGGL((wave_span<K, true>), dim3((unsigned)((NPX / (64 * K) + 3) / 4)), dim3(256), 0, 0, o); }, iters)); \
    rep("wave_span K=" #K " cached", time_it([&] { hipLaunchKernelGGL((wave_span<K, false>), dim3((unsigned)((NPX / (64 * K) + 3) / 4)), dim3(256), 0, 0, o); }, iters));
    SPAN(2) SPAN(4) SPAN(8) SPAN(16)
    for (int g : {1024, 2048, 4096, 8192, 16384}) {
        char name[64];
        snprintf(name, sizeof name, "grid_stride G=%d nt", g);
        rep(name, time_it([&] { hipLaunchKernelGGL(grid_stride<true>, dim3(g), dim3(256), 0, 0, o); }, iters));
        snprintf(name, sizeof name, "grid_stride G=%d cached", g);
        rep(name, time_it([&] { hipLaunchKernelGGL(grid_stride<false>, dim3(g), dim3(256), 0, 0, o); }, iters));
    }
    rep("hipMemsetD32Async", time_it([&] { hipMemsetD32Async((hipDeviceptr_t)o, 0x3e4ccccd, NPX * 4, 0); }, iters));
    hipFree(o);
    return 0;
}
