// rtm_internal.h — what rtm_group.cpp (the RCCL multi-GPU frame) needs from the
// single-device library (rtm_api.cpp) beyond the public C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rtm.h"

namespace rtm {
namespace internal {

// Validate a frame's inputs as every render entry point does (rtm_last_error set on failure).
int check_frame(const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow, int32_t width,
                int32_t height, int32_t march_steps, int32_t flags);
// bytes per pixel of an RTM_FORMAT_* (0: unknown)
int32_t bytes_per_pixel(int32_t format);
// set rtm_last_error and return code
int set_error(int code, const char* msg);
int ctx_device(const rtm_ctx* ctx);
hipStream_t ctx_stream(const rtm_ctx* ctx);

}  // namespace internal
}  // namespace rtm
