// Map-store probe (diagnostic, not part of the library): the HBM write counters of a
// coded shadow map (1 B per texel, 128 x 4 blocks of 512 B, rtm_kernels.h
// smap_code_index) written in the coded tile's shape -- a wave per 128 x 16 strip,
// one 8-byte store per lane per block (global_store_dwordx2) -- against the same bytes
// stored 16 B per lane.  Eight 3840x2160 maps per launch (66.4 MB), as a batched shadow
// pass writes them.  hipcc --offload-arch=gfx950 -O3 map_store_probe.hip -o map_store_probe
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int W = 3840, H = 2160, NF = 8;
constexpr int BW = W / 128;                  // blocks per block row
constexpr size_t MAP = (size_t)W * H;        // bytes per map

// the coded tile's store: lane l of the wave covering rows [y0, y0+16) writes the 8 bytes
// of its 2 columns x 4 rows of each of the 4 blocks
__global__ __launch_bounds__(256) void store8(unsigned char* __restrict__ map) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int y0 = (blockIdx.y * 4 + wv) * 16;
    unsigned char* m = map + (size_t)blockIdx.z * MAP;
    if (y0 >= H) return;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const size_t blk = (size_t)((y0 >> 2) + b) * BW + blockIdx.x;
        *reinterpret_cast<uint2*>(m + blk * 512 + lane * 8) = make_uint2(0x01020304u + b, 0x05060708u + lane);
    }
}

// the same blocks, 16 B per lane: lanes 0-31 write block 2b, lanes 32-63 block 2b+1
__global__ __launch_bounds__(256) void store16(unsigned char* __restrict__ map) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int y0 = (blockIdx.y * 4 + wv) * 16;
    unsigned char* m = map + (size_t)blockIdx.z * MAP;
    if (y0 >= H) return;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int b = 2 * h + (lane >> 5);
        const size_t blk = (size_t)((y0 >> 2) + b) * BW + blockIdx.x;
        *reinterpret_cast<uint4*>(m + blk * 512 + (lane & 31) * 16) = make_uint4(b, lane, 3u, 4u);
    }
}

int main() {
    unsigned char* map;
    if (hipMalloc(&map, MAP * NF) != hipSuccess) return 1;
    dim3 g(BW, (H + 63) / 64, NF);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int v = 0; v < 2; ++v) {
        for (int it = 0; it < 3; ++it) {  // warm
            if (v == 0) hipLaunchKernelGGL(store8, g, dim3(256), 0, 0, map);
            else hipLaunchKernelGGL(store16, g, dim3(256), 0, 0, map);
        }
        hipEventRecord(e0);
        const int reps = 20;
        for (int it = 0; it < reps; ++it) {
            if (v == 0) hipLaunchKernelGGL(store8, g, dim3(256), 0, 0, map);
            else hipLaunchKernelGGL(store16, g, dim3(256), 0, 0, map);
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%s: %.2f us per launch, %.2f TB/s (%zu bytes per launch)\n", v ? "store16" : "store8",
               ms * 1e3f / reps, (double)MAP * NF / (ms * 1e-3 / reps) / 1e12, MAP * NF);
    }
    hipFree(map);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
