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
// A frame's inputs validated and precomputed once (FrameArgs + device tables),
// then enqueued per row band on any context without repeating the host work.
struct PreparedFrame;
PreparedFrame* new_prepared();
void delete_prepared(PreparedFrame* f);
int prepare_frame(PreparedFrame* f, const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow,
                  int32_t width, int32_t height, int32_t march_steps, int32_t flags);
// Cyclic row stripes (the multi-GPU frame's balanced partition): a launch of local
// rows [0, rows) renders image row phase + (j / stripe_rows) * stride + j % stripe_rows
// for local row j (rows past H skipped); out_global: the output buffer is the whole
// image (rows land at their image rows), else the launch's compact rows.
struct RowMap {
    int32_t stripe_rows = 0, stride = 0, phase = 0, out_global = 0;
};
// image rows of rank r of n under S-row cyclic stripes (the local row count)
int32_t stripe_rows_of(int32_t H, int32_t n, int32_t S, int32_t r);
// rows [row_begin, row_end) in `format` into out_dev, on ctx's stream (map: stripes,
// row_begin = 0 and row_end = the local row count then)
int enqueue_prepared(rtm_ctx* ctx, const PreparedFrame* f, int32_t format, int32_t row_begin, int32_t row_end,
                     void* out_dev, const RowMap* map = nullptr, int lane = 0);
// n frames' rows [row_begin, row_end) in `format`, frame k into outs[k], on the stream
// of ctx's lane `lane` (0: ctx's own stream; lanes_begin forks the others): one launch
// per pass when the frames share their march tables (rtm_ctx_set_batch's batched
// kernels), else frame by frame
int enqueue_prepared_batch(rtm_ctx* ctx, const PreparedFrame* const* fs, int n, int32_t format, int32_t row_begin,
                           int32_t row_end, void* const* outs, const RowMap* map = nullptr, int lane = 0);
// Lanes for n_batches batches of width x rows frames (the rtm_render_frames_async
// rule, rtm_ctx_set_lanes honoured): creates them and makes them start after ctx's
// stream; returns the count (1: ctx's stream only) or a negative error.
// max_lanes > 0 caps the count (1: the caller's batches must run in order).
int lanes_begin(rtm_ctx* ctx, int32_t width, int32_t rows, int32_t n_batches, int32_t max_lanes = 0);
// the count lanes_begin would return, without creating or forking anything
int lanes_plan(const rtm_ctx* ctx, int32_t width, int32_t rows, int32_t n_batches);
// ctx's stream waits for lanes 1..L-1 (every batch enqueued on them is then in its order)
int lanes_end(rtm_ctx* ctx, int L);
// the stream of ctx's lane (0: ctx's own)
hipStream_t lane_stream(const rtm_ctx* ctx, int lane);
// frames per launch the library's auto rule picks for width x rows frames
int auto_frames_per_launch(int32_t width, int32_t rows);
// bytes per pixel of an RTM_FORMAT_* (0: unknown)
int32_t bytes_per_pixel(int32_t format);
// set rtm_last_error and return code
int set_error(int code, const char* msg);
int ctx_device(const rtm_ctx* ctx);
hipStream_t ctx_stream(const rtm_ctx* ctx);

}  // namespace internal
}  // namespace rtm
