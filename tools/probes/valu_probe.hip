// VALU throughput probe (diagnostic): f32 vs f64 FMA/add/mul with 8 independent
// chains per lane, 256-thread blocks, 8 waves/SIMD worth of blocks.
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T, int OP>  // OP 0 fma, 1 add, 2 mul
__global__ void chains(T* out, T seed, int iters) {
    T v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = seed + (T)(threadIdx.x + j);
    const T m = (T)1.0000001, c = (T)1e-7;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (OP == 0) v[j] = __builtin_fma(v[j], m, c);
            else if (OP == 1) v[j] = v[j] + c;
            else v[j] = v[j] * m;
        }
    }
    T s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j];
    if (s == (T)-1) out[threadIdx.x] = s;
}

template <typename T, int OP>
static void run(const char* name, T* out) {
    const int blocks = 256 * 8, iters = 4096;  // 8 WGs of 4 waves per CU = 8 waves/SIMD
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL((chains<T, OP>), dim3(blocks), dim3(256), 0, 0, out, (T)1, iters);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((chains<T, OP>), dim3(blocks), dim3(256), 0, 0, out, (T)1, iters);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double lane_ops = (double)blocks * 256 * iters * 8;
    const double wave_instr_per_simd = lane_ops / 64 / 1024;
    printf("%-10s %8.3f ms  %7.2f T lane-ops/s  %5.2f cycles per wave-instruction per SIMD at 2.4 GHz\n", name, ms,
           lane_ops / (ms * 1e-3) / 1e12, ms * 1e-3 * 2.4e9 / wave_instr_per_simd);
}

int main() {
    void* out;
    if (hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
    run<float, 0>("f32 fma", (float*)out);
    run<float, 1>("f32 add", (float*)out);
    run<double, 0>("f64 fma", (double*)out);
    run<double, 1>("f64 add", (double*)out);
    run<double, 2>("f64 mul", (double*)out);
    return 0;
}
