// rtm_encode.h — writeColorImage (main.rs:660-704) launchers.
#pragma once

#include <stdint.h>

#include "../../include/rtm.h"

namespace rtm {

// The encode is a monotone step function of the clamped f32 channel value v
// (tests/test_encode.py proves it over every f32 in [0,1]), described exactly by
//   t[k]      = smallest f32 v in [0,1] whose byte is >= k (t[0] = 0)
//   bucket[i] = byte of the smallest v whose bit pattern is in [i<<16, (i+1)<<16)
// both built on the host with the platform powf.  A 2^16-ulp bucket never spans
// more than one threshold (checked when the table is built), so a byte is
// bucket[bits>>16] plus at most one compare against t.
constexpr int ENC_BUCKET_SHIFT = 16;
constexpr int ENC_BUCKETS = (0x3F800000 >> ENC_BUCKET_SHIFT) + 1;  // 16257

struct EncodeTable {
    float t[256];
    uint8_t bucket[ENC_BUCKETS];
    int32_t max_crossings;  // thresholds inside one bucket (1 for libm powf)
};

// Device copy: t at offset 0 (1 KiB), bucket at offset 1024.
constexpr size_t ENC_DEV_BYTES = 1024 + ENC_BUCKETS;

// rgba must be 16-byte aligned (float4 loads); rgb any alignment.
int launch_encode_rgb8(const float* rgba, int64_t n, uint8_t* rgb, const void* tab_dev, void* stream);
// rowlen/rowoff: H int64 each; total: 1 int64 (= header_len + text length).
// out == nullptr: lengths and offsets only.
int launch_ppm_text(const uint8_t* rgb, int W, int H, int64_t header_len, int64_t* rowlen, int64_t* rowoff,
                    int64_t* total, char* out, void* stream);

}  // namespace rtm
