// rtm_encode.hip — writeColorImage (main.rs:660-704) on the GPU: the RGB8 pixel
// encode and the PPM "P3" text, from a device RGBA f32 framebuffer.
//
// Per channel the reference computes (f32 throughout, main.rs:674-684):
//     v = c.max(0.0).min(1.0);  v = f32::powf(v, 1.0/2.2);  byte = (v * 255.0) as i64
// v -> byte is a monotone step function of v with 256 levels (proved over every
// f32 in [0,1] by tests/test_encode.py), so it is fully described by its 255
// thresholds.  The host library finds them with the platform powf (the libm the
// Rust binary calls); the kernels look v up among them: bit-identical to
// per-pixel powf, with no transcendental on the GPU.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rtm_encode.h"

namespace rtm {

namespace {

constexpr int EBLOCK = 256;
constexpr int PPT = 4;                   // pixels per thread
constexpr int CHUNK = EBLOCK * PPT;      // pixels per PPM chunk
constexpr int PIX_TEXT_MAX = 13;         // "255 255 255  "

// byte for one channel.  Clamp as f32::max(0.0) / f32::min(1.0): NaN -> 0.0, and
// -0.0 -> +0.0 (both encode to 0), so v's bits are in [0, 0x3F800000].  The
// bucket gives the byte of the bucket's first value; the loop adds the (at most
// one, host-checked) threshold inside the bucket and stays exact even if the
// table were coarser.
__device__ __forceinline__ uint32_t enc_channel(float c, const float* __restrict__ T,
                                                const uint8_t* __restrict__ B) {
    float v = c > 0.0f ? c : 0.0f;
    v = v < 1.0f ? v : 1.0f;
    uint32_t k = B[__float_as_uint(v) >> ENC_BUCKET_SHIFT];
    while (k < 255u && v >= T[k + 1]) ++k;
    return k;
}

__device__ __forceinline__ uint32_t enc3(const float4& p, const float* T, const uint8_t* B) {
    return enc_channel(p.x, T, B) | (enc_channel(p.y, T, B) << 8) | (enc_channel(p.z, T, B) << 16);
}

// Four pixels per thread: four 16-byte loads, twelve output bytes packed into
// three little-endian dwords (ALIGNED: rgb is 4-byte aligned, dword stores;
// otherwise byte stores).  The n % 4 tail pixels go through the byte path.
template <bool ALIGNED>
__global__ __launch_bounds__(EBLOCK) void encode_rgb8_kernel(const float4* __restrict__ rgba, int64_t n,
                                                             uint8_t* __restrict__ rgb, const float* __restrict__ T,
                                                             const uint8_t* __restrict__ B) {
    const int64_t nq = n >> 2;
    const int64_t stride = (int64_t)gridDim.x * EBLOCK;
    for (int64_t q = (int64_t)blockIdx.x * EBLOCK + threadIdx.x; q < nq; q += stride) {
        const float4 p0 = rgba[4 * q + 0], p1 = rgba[4 * q + 1], p2 = rgba[4 * q + 2], p3 = rgba[4 * q + 3];
        const uint32_t a = enc3(p0, T, B), b = enc3(p1, T, B), c = enc3(p2, T, B), d = enc3(p3, T, B);
        const uint32_t w0 = a | (b << 24);
        const uint32_t w1 = (b >> 8) | (c << 16);
        const uint32_t w2 = (c >> 16) | (d << 8);
        if (ALIGNED) {
            uint32_t* o = reinterpret_cast<uint32_t*>(rgb + 12 * q);
            o[0] = w0;
            o[1] = w1;
            o[2] = w2;
        } else {
            uint8_t* o = rgb + 12 * q;
            const uint32_t w[3] = {w0, w1, w2};
#pragma unroll
            for (int i = 0; i < 12; ++i) o[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
        }
    }
    for (int64_t i = 4 * nq + (int64_t)blockIdx.x * EBLOCK + threadIdx.x; i < n; i += stride) {
        const uint32_t a = enc3(rgba[i], T, B);
        rgb[3 * i + 0] = (uint8_t)a;
        rgb[3 * i + 1] = (uint8_t)(a >> 8);
        rgb[3 * i + 2] = (uint8_t)(a >> 16);
    }
}

__device__ __forceinline__ int ndigits(uint32_t v) { return v >= 100 ? 3 : (v >= 10 ? 2 : 1); }

// Text of one pixel: format!("{} {} {}  ", r, g, b) (main.rs:684).
__device__ __forceinline__ int pixel_len(uint32_t r, uint32_t g, uint32_t b) {
    return ndigits(r) + ndigits(g) + ndigits(b) + 4;
}

__device__ __forceinline__ char* put_num(char* o, uint32_t v) {
    if (v >= 100) *o++ = (char)('0' + v / 100);
    if (v >= 10) *o++ = (char)('0' + (v / 10) % 10);
    *o++ = (char)('0' + v % 10);
    return o;
}

// Row lengths: one block per row; row text = pixels + '\n' (main.rs:687).
__global__ __launch_bounds__(EBLOCK) void ppm_row_len_kernel(const uint8_t* __restrict__ rgb, int W,
                                                             int64_t* __restrict__ rowlen) {
    __shared__ int64_t part[EBLOCK];
    const int y = blockIdx.x;
    const uint8_t* row = rgb + 3 * (int64_t)y * W;
    int64_t s = 0;
    for (int x = threadIdx.x; x < W; x += EBLOCK) s += pixel_len(row[3 * x], row[3 * x + 1], row[3 * x + 2]);
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = EBLOCK / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) part[threadIdx.x] += part[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) rowlen[y] = part[0] + 1;
}

// Exclusive scan of the H row lengths in one block (H <= RTM_MAX_DIM).
__global__ __launch_bounds__(EBLOCK) void ppm_row_scan_kernel(const int64_t* __restrict__ rowlen, int H,
                                                              int64_t base, int64_t* __restrict__ rowoff,
                                                              int64_t* __restrict__ total) {
    __shared__ int64_t part[EBLOCK];
    const int per = (H + EBLOCK - 1) / EBLOCK;
    const int b = threadIdx.x * per;
    int64_t s = 0;
    for (int i = 0; i < per && b + i < H; ++i) s += rowlen[b + i];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {  // 256 partial sums: a short serial scan
        int64_t run = base;
        for (int i = 0; i < EBLOCK; ++i) {
            const int64_t v = part[i];
            part[i] = run;
            run += v;
        }
        *total = run;
    }
    __syncthreads();
    int64_t run = part[threadIdx.x];
    for (int i = 0; i < per && b + i < H; ++i) {
        rowoff[b + i] = run;
        run += rowlen[b + i];
    }
}

// Write the text: one block per row, CHUNK pixels at a time (PPT consecutive
// pixels per thread).  A block-wide exclusive scan of the per-thread text
// lengths places each thread's text in an LDS staging buffer; the chunk is then
// copied out with coalesced dword stores (byte stores only for the unaligned
// head and tail).  `out` is 4-byte aligned.
__global__ __launch_bounds__(EBLOCK) void ppm_write_kernel(const uint8_t* __restrict__ rgb, int W,
                                                           const int64_t* __restrict__ rowoff,
                                                           char* __restrict__ out) {
    __shared__ int scan[EBLOCK];
    __shared__ char buf[CHUNK * PIX_TEXT_MAX + 4];
    const int y = blockIdx.x;
    const int t = threadIdx.x;
    const uint8_t* row = rgb + 3 * (int64_t)y * W;
    int64_t pos = rowoff[y];
    for (int x0 = 0; x0 < W; x0 += CHUNK) {
        const int xs = x0 + t * PPT;
        const int np = W - xs < 0 ? 0 : (W - xs > PPT ? PPT : W - xs);
        uint32_t px[PPT][3];
        int len = 0;
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
            if (i < np) {
                px[i][0] = row[3 * (xs + i)];
                px[i][1] = row[3 * (xs + i) + 1];
                px[i][2] = row[3 * (xs + i) + 2];
                len += pixel_len(px[i][0], px[i][1], px[i][2]);
            }
        }
        scan[t] = len;
        __syncthreads();
        for (int off = 1; off < EBLOCK; off <<= 1) {  // Hillis-Steele inclusive scan
            const int v = t >= off ? scan[t - off] : 0;
            __syncthreads();
            scan[t] += v;
            __syncthreads();
        }
        const int chunk = scan[EBLOCK - 1];
        char* o = buf + (scan[t] - len);
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
            if (i < np) {
                o = put_num(o, px[i][0]);
                *o++ = ' ';
                o = put_num(o, px[i][1]);
                *o++ = ' ';
                o = put_num(o, px[i][2]);
                *o++ = ' ';
                *o++ = ' ';
            }
        }
        __syncthreads();
        const int head = min((int)((4 - (pos & 3)) & 3), chunk);
        if (t < head) out[pos + t] = buf[t];
        const int nw = (chunk - head) >> 2;
        uint32_t* ow = reinterpret_cast<uint32_t*>(out + pos + head);
        for (int j = t; j < nw; j += EBLOCK) {
            const char* c = buf + head + 4 * j;
            ow[j] = (uint32_t)(uint8_t)c[0] | ((uint32_t)(uint8_t)c[1] << 8) | ((uint32_t)(uint8_t)c[2] << 16) |
                    ((uint32_t)(uint8_t)c[3] << 24);
        }
        const int done = head + 4 * nw;
        if (t < chunk - done) out[pos + done + t] = buf[done + t];
        pos += chunk;
        __syncthreads();
    }
    if (t == 0) out[pos] = '\n';
}

inline int ok() { return hipGetLastError() == hipSuccess ? 0 : RTM_ERR_HIP; }

}  // namespace

int launch_encode_rgb8(const float* rgba, int64_t n, uint8_t* rgb, const void* tab_dev, void* stream) {
    if (n <= 0) return 0;
    const float* T = static_cast<const float*>(tab_dev);
    const uint8_t* B = static_cast<const uint8_t*>(tab_dev) + 1024;
    int64_t blocks = ((n >> 2) + EBLOCK - 1) / EBLOCK;
    if (blocks < 1) blocks = 1;
    if (blocks > 16384) blocks = 16384;
    const float4* p = reinterpret_cast<const float4*>(rgba);
    if (((uintptr_t)rgb & 3) == 0)
        hipLaunchKernelGGL(encode_rgb8_kernel<true>, dim3((unsigned)blocks), dim3(EBLOCK), 0, (hipStream_t)stream,
                           p, n, rgb, T, B);
    else
        hipLaunchKernelGGL(encode_rgb8_kernel<false>, dim3((unsigned)blocks), dim3(EBLOCK), 0, (hipStream_t)stream,
                           p, n, rgb, T, B);
    return ok();
}

int launch_ppm_text(const uint8_t* rgb, int W, int H, int64_t header_len, int64_t* rowlen, int64_t* rowoff,
                    int64_t* total, char* out, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(ppm_row_len_kernel, dim3((unsigned)H), dim3(EBLOCK), 0, s, rgb, W, rowlen);
    hipLaunchKernelGGL(ppm_row_scan_kernel, dim3(1), dim3(EBLOCK), 0, s, rowlen, H, header_len, rowoff, total);
    if (out) hipLaunchKernelGGL(ppm_write_kernel, dim3((unsigned)H), dim3(EBLOCK), 0, s, rgb, W, rowoff, out);
    return ok();
}

}  // namespace rtm
