// rtm_group.cpp — the north star's multi-GPU frame (BASELINE.json north_star,
// SURVEY.md §8e): the image tile-partitioned into row bands over N devices and
// assembled in the root's device buffer by ONE RCCL gather over xGMI.
//
// The reference renders one Map2d<Color32> frame on one CPU thread
// (renderColorImage, main.rs:709-716, 896-898); nothing in it is distributed.
// Every pixel is independent, so a band needs no other band's data except
// shadow texels, which each band evaluates itself (RTM_FLAG_FUSED_SHADOW, the
// same image bits).  The one exchange is the final gather.
//
// RCCL is loaded at run time (dlopen "librccl.so.1": the copy torch.distributed
// already mapped when the process has one, so the process holds one RCCL), so
// librtm.so itself does not depend on it: single-device callers never load it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "rtm_internal.h"

using rtm::internal::set_error;

namespace {

// ---- RCCL entry points (rccl.h) resolved from the shared library ----
struct Rccl {
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
    ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
    std::string error;  // empty: loaded
};

const Rccl& rccl() {
    static const Rccl r = [] {
        Rccl x;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = dlerror();
            x.error = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
            return x;
        }
        bool ok = true;
        auto sym = [&](const char* name) {
            void* p = dlsym(h, name);
            if (!p) {
                ok = false;
                x.error = std::string("librccl.so.1 lacks ") + name;
            }
            return p;
        };
        x.GetUniqueId = reinterpret_cast<decltype(x.GetUniqueId)>(sym("ncclGetUniqueId"));
        x.CommInitRank = reinterpret_cast<decltype(x.CommInitRank)>(sym("ncclCommInitRank"));
        x.CommInitAll = reinterpret_cast<decltype(x.CommInitAll)>(sym("ncclCommInitAll"));
        x.CommDestroy = reinterpret_cast<decltype(x.CommDestroy)>(sym("ncclCommDestroy"));
        x.CommAbort = reinterpret_cast<decltype(x.CommAbort)>(sym("ncclCommAbort"));
        x.CommGetAsyncError = reinterpret_cast<decltype(x.CommGetAsyncError)>(sym("ncclCommGetAsyncError"));
        x.Send = reinterpret_cast<decltype(x.Send)>(sym("ncclSend"));
        x.Recv = reinterpret_cast<decltype(x.Recv)>(sym("ncclRecv"));
        x.GroupStart = reinterpret_cast<decltype(x.GroupStart)>(sym("ncclGroupStart"));
        x.GroupEnd = reinterpret_cast<decltype(x.GroupEnd)>(sym("ncclGroupEnd"));
        x.GetErrorString = reinterpret_cast<decltype(x.GetErrorString)>(sym("ncclGetErrorString"));
        if (!ok) x.GetErrorString = nullptr;
        return x;
    }();
    return r;
}

int comm_fail(const char* what, ncclResult_t r) {
    char buf[256];
    const Rccl& R = rccl();
    snprintf(buf, sizeof buf, "%s: %s", what, R.GetErrorString ? R.GetErrorString(r) : "RCCL error");
    return set_error(RTM_ERR_COMM, buf);
}

int hip_fail(const char* what, hipError_t e) {
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    return set_error(RTM_ERR_HIP, buf);
}

#define NCCL_TRY(expr)                                   \
    do {                                                 \
        ncclResult_t r_ = (expr);                        \
        if (r_ != ncclSuccess) return comm_fail(#expr, r_); \
    } while (0)
#define GHIP_TRY(expr)                                  \
    do {                                                \
        hipError_t e_ = (expr);                         \
        if (e_ != hipSuccess) return hip_fail(#expr, e_); \
    } while (0)

struct Guard {  // current device for a scope
    int prev = 0;
    explicit Guard(int dev) {
        (void)hipGetDevice(&prev);
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~Guard() { (void)hipSetDevice(prev); }
};

// Row band of rank r among n (N bands of ceil(H/N) rows; the last
// ones may be short or empty when N does not divide H).  shard.py row_band mirrors it.
inline void band_rows(int32_t H, int32_t n, int32_t r, int32_t* r0, int32_t* r1) {
    const int32_t band = (H + n - 1) / n;
    *r0 = std::min<int64_t>(H, (int64_t)r * band);
    *r1 = std::min<int64_t>(H, (int64_t)(r + 1) * band);
}

// The partition's default stripe height: 8-row cyclic stripes once there are several
// ranks (a function of the rank count only, so every rank of a one-process-per-GPU
// group picks the same; rtm_group_set_partition is collective).  Contiguous bands of
// ceil(H/N) rows were measured 1.26-1.56x max/mean band time at N = 4-8 (the spheres
// sit mid-frame, and a band's cost follows its hit pixels); 8-row stripes model at
// 1.01-1.06 (tools/band_balance.py, profiles/r03_band_balance.json).
int32_t default_stripe(int32_t n) { return n > 1 ? 8 : 0; }

// Rank r's rows of an H-row frame: contiguous [r0, r0 + rows) or S-row cyclic stripes
// (local row j = image row r*S + (j / S)*N*S + j % S).
struct Part {
    int32_t rows = 0, r0 = 0;
    rtm::internal::RowMap map;
};

Part part_of(int32_t H, int32_t n, int32_t S, int32_t r) {
    Part p;
    if (S > 0 && n > 1) {
        p.rows = rtm::internal::stripe_rows_of(H, n, S, r);
        p.map.stripe_rows = S;
        p.map.stride = n * S;
        p.map.phase = r * S;
    } else {
        int32_t r1;
        band_rows(H, n, r, &p.r0, &r1);
        p.rows = r1 - p.r0;
    }
    return p;
}

// Place a part's compact rows (src) at their image rows of the frame dst: one copy for
// a contiguous band, a 2-D copy (S rows per stripe, pitch N*S rows) plus the short
// tail stripe for stripes.
hipError_t place_rows(void* dst, const void* src, const Part& p, size_t row_bytes, hipMemcpyKind kind,
                      hipStream_t s) {
    if (p.rows <= 0) return hipSuccess;
    if (p.map.stripe_rows <= 0)
        return hipMemcpyAsync((char*)dst + row_bytes * (size_t)p.r0, src, row_bytes * (size_t)p.rows, kind, s);
    const int32_t S = p.map.stripe_rows, full = p.rows / S, tail = p.rows % S;
    char* d0 = (char*)dst + row_bytes * (size_t)p.map.phase;
    hipError_t e = hipSuccess;
    if (full > 0)
        e = hipMemcpy2DAsync(d0, row_bytes * (size_t)p.map.stride, src, row_bytes * (size_t)S, row_bytes * (size_t)S,
                             (size_t)full, kind, s);
    if (e == hipSuccess && tail > 0)
        e = hipMemcpyAsync(d0 + row_bytes * (size_t)p.map.stride * (size_t)full,
                           (const char*)src + row_bytes * (size_t)S * (size_t)full, row_bytes * (size_t)tail, kind, s);
    return e;
}

}  // namespace

// One local device of the group.  A chunk of frames renders into one of its staging
// slots (chunks spread over the context's L lanes: L + 1 slots, at most NSLOT, keep
// every lane busy while a chunk is in transfer); a slot is reused once its sends have
// read it.
constexpr int NSLOT = 4;
struct Member {
    rtm_ctx* ctx = nullptr;
    int device = 0;
    int rank = 0;
    ncclComm_t comm = nullptr;
    hipStream_t xfer = nullptr;      // the member's RCCL transfers
    hipEvent_t start = nullptr;      // frame start on the render stream (the root's receives wait for it)
    hipEvent_t ready[NSLOT] = {};    // band rendered into stage[s]
    hipEvent_t sent[NSLOT] = {};     // stage[s] read by its send
    hipEvent_t done = nullptr;       // the frame's transfers on this member are finished
    hipEvent_t lb_sent = nullptr;    // loopback transport: this member's send is posted
    hipEvent_t lb_recv = nullptr;    // loopback transport: the root's copy of it has run
    void* stage[NSLOT] = {};
    size_t stage_bytes = 0;
    int nstage = 0;  // staging slots allocated (stage[0 .. nstage))
    int slot = 0;
};

struct rtm_group {
    int32_t n_ranks = 0;
    std::vector<Member> m;
    bool aborted = false;
    bool root_staging = false;
    bool loopback = false;     // transport: device copies on the root's stream instead of RCCL
    bool host_direct = false;  // rtm_group_render: every band straight to the host, no gather
    int32_t stripe = -1;       // partition: S-row cyclic stripes (S > 0) or contiguous bands (0); -1: default
    void* recv = nullptr;      // the root's receive staging for striped RCCL gathers (n_ranks parts)
    size_t recv_bytes = 0;
    int recv_device = 0;
    void* root_frame = nullptr;  // rtm_group_render: the assembled frame on the root's device
    size_t root_frame_bytes = 0;
};

namespace {

void release(rtm_group* g, bool destroy_comms) {
    const Rccl& R = rccl();
    for (Member& mb : g->m) {
        Guard d(mb.device);
        // renders (which write the staging slots) and transfers (which read them) first
        if (mb.ctx) (void)rtm_ctx_synchronize(mb.ctx);
        if (mb.xfer) (void)hipStreamSynchronize(mb.xfer);
        if (mb.comm && destroy_comms && R.CommDestroy) (void)R.CommDestroy(mb.comm);
        mb.comm = nullptr;
        for (hipEvent_t* e : {&mb.start, &mb.done, &mb.lb_sent, &mb.lb_recv})
            if (*e) {
                (void)hipEventDestroy(*e);
                *e = nullptr;
            }
        for (int k = 0; k < NSLOT; ++k)
            for (hipEvent_t* e : {&mb.ready[k], &mb.sent[k]})
                if (*e) {
                    (void)hipEventDestroy(*e);
                    *e = nullptr;
                }
        for (void*& p : mb.stage)
            if (p) {
                (void)hipFree(p);
                p = nullptr;
            }
        if (mb.xfer) (void)hipStreamDestroy(mb.xfer);
        mb.xfer = nullptr;
        if (mb.ctx) rtm_ctx_destroy(mb.ctx);
        mb.ctx = nullptr;
    }
    if (g->root_frame) {
        for (Member& mb : g->m)
            if (mb.rank == 0) {
                Guard d(mb.device);
                (void)hipFree(g->root_frame);
            }
        g->root_frame = nullptr;
        g->root_frame_bytes = 0;
    }
    if (g->recv) {
        Guard d(g->recv_device);
        (void)hipFree(g->recv);
        g->recv = nullptr;
        g->recv_bytes = 0;
    }
}

// Contexts, transfer streams and events of the members (comms set by the caller).
int setup_members(rtm_group* g) {
    for (Member& mb : g->m) {
        int rc = rtm_ctx_create(mb.device, &mb.ctx);
        if (rc) return rc;
        Guard d(mb.device);
        GHIP_TRY(hipStreamCreateWithFlags(&mb.xfer, hipStreamNonBlocking));
        for (hipEvent_t* e : {&mb.start, &mb.done, &mb.lb_sent, &mb.lb_recv})
            GHIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
        for (int k = 0; k < NSLOT; ++k)
            for (hipEvent_t* e : {&mb.ready[k], &mb.sent[k]}) GHIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    return RTM_OK;
}

// At least `nslot` staging slots of at least `bytes` each (slots only grow: a slot in
// the rotation stays valid).  At 7680x4320 RGBA f32 and N = 2 a slot of 2 frames'
// parts is 0.53 GB, so a one-lane member keeps 2 slots, not NSLOT.
int ensure_stage(Member& mb, size_t bytes, int nslot) {
    nslot = std::max(1, std::min(nslot, NSLOT));
    if (bytes <= mb.stage_bytes && nslot <= mb.nstage) return RTM_OK;
    bytes = std::max(bytes, mb.stage_bytes);
    nslot = std::max(nslot, mb.nstage);
    Guard d(mb.device);
    // the staging buffers are idle once their renders and their last sends are done
    GHIP_TRY(hipStreamSynchronize(rtm::internal::ctx_stream(mb.ctx)));
    GHIP_TRY(hipStreamSynchronize(mb.xfer));
    for (void*& p : mb.stage) {
        if (p) (void)hipFree(p);
        p = nullptr;
    }
    mb.stage_bytes = 0;
    mb.nstage = 0;
    mb.slot = 0;
    for (int k = 0; k < nslot; ++k)
        if (hipMalloc(&mb.stage[k], bytes) != hipSuccess) return set_error(RTM_ERR_OOM, "band staging allocation failed");
    mb.stage_bytes = bytes;
    mb.nstage = nslot;
    return RTM_OK;
}

}  // namespace

extern "C" {

int rtm_group_unique_id(uint8_t id[128]) {
    if (!id) return set_error(RTM_ERR_INVALID, "id is NULL");
    const Rccl& R = rccl();
    if (!R.error.empty()) return set_error(RTM_ERR_COMM, R.error.c_str());
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId u;
    NCCL_TRY(R.GetUniqueId(&u));
    std::memcpy(id, &u, sizeof u);
    return RTM_OK;
}

int rtm_group_create(int32_t n_devices, const int32_t* devices, rtm_group** out) {
    if (!out) return set_error(RTM_ERR_INVALID, "out is NULL");
    *out = nullptr;
    const int nd = rtm_device_count();
    if (nd <= 0) return set_error(RTM_ERR_NO_DEVICE, "no HIP device visible");
    if (n_devices < 1 || n_devices > nd) return set_error(RTM_ERR_INVALID, "n_devices outside [1, device count]");
    std::vector<int> dev((size_t)n_devices);
    for (int i = 0; i < n_devices; ++i) {
        dev[(size_t)i] = devices ? devices[i] : i;
        if (dev[(size_t)i] < 0 || dev[(size_t)i] >= nd) return set_error(RTM_ERR_INVALID, "device id out of range");
        for (int j = 0; j < i; ++j)
            if (dev[(size_t)j] == dev[(size_t)i]) return set_error(RTM_ERR_INVALID, "a device appears twice");
    }
    const Rccl& R = rccl();
    if (!R.error.empty()) return set_error(RTM_ERR_COMM, R.error.c_str());
    std::unique_ptr<rtm_group> g(new rtm_group);
    g->n_ranks = n_devices;
    g->m.resize((size_t)n_devices);
    for (int i = 0; i < n_devices; ++i) {
        g->m[(size_t)i].device = dev[(size_t)i];
        g->m[(size_t)i].rank = i;
    }
    int rc = setup_members(g.get());
    if (rc) {
        release(g.get(), false);
        return rc;
    }
    std::vector<ncclComm_t> comms((size_t)n_devices, nullptr);
    ncclResult_t r = R.CommInitAll(comms.data(), n_devices, dev.data());  // rccl.h:236
    if (r != ncclSuccess) {
        release(g.get(), false);
        return comm_fail("ncclCommInitAll", r);
    }
    for (int i = 0; i < n_devices; ++i) g->m[(size_t)i].comm = comms[(size_t)i];
    *out = g.release();
    return RTM_OK;
}

int rtm_group_create_loopback(int32_t n_members, const int32_t* devices, rtm_group** out) {
    if (!out) return set_error(RTM_ERR_INVALID, "out is NULL");
    *out = nullptr;
    const int nd = rtm_device_count();
    if (nd <= 0) return set_error(RTM_ERR_NO_DEVICE, "no HIP device visible");
    if (n_members < 1 || n_members > 64) return set_error(RTM_ERR_INVALID, "n_members outside [1, 64]");
    std::unique_ptr<rtm_group> g(new rtm_group);
    g->n_ranks = n_members;
    g->loopback = true;
    g->m.resize((size_t)n_members);
    for (int i = 0; i < n_members; ++i) {
        const int d = devices ? devices[i] : 0;
        if (d < 0 || d >= nd) return set_error(RTM_ERR_INVALID, "device id out of range");
        g->m[(size_t)i].device = d;
        g->m[(size_t)i].rank = i;
    }
    int rc = setup_members(g.get());
    if (rc) {
        release(g.get(), false);
        return rc;
    }
    *out = g.release();
    return RTM_OK;
}

int rtm_group_create_rank(int32_t device, int32_t n_ranks, int32_t rank, const uint8_t id[128], rtm_group** out) {
    if (!out || !id) return set_error(RTM_ERR_INVALID, "out/id is NULL");
    *out = nullptr;
    const int nd = rtm_device_count();
    if (nd <= 0) return set_error(RTM_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= nd) return set_error(RTM_ERR_INVALID, "device out of range");
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks) return set_error(RTM_ERR_INVALID, "rank outside [0, n_ranks)");
    const Rccl& R = rccl();
    if (!R.error.empty()) return set_error(RTM_ERR_COMM, R.error.c_str());
    std::unique_ptr<rtm_group> g(new rtm_group);
    g->n_ranks = n_ranks;
    g->m.resize(1);
    g->m[0].device = device;
    g->m[0].rank = rank;
    int rc = setup_members(g.get());
    if (rc) {
        release(g.get(), false);
        return rc;
    }
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    ncclComm_t c = nullptr;
    ncclResult_t r;
    {
        Guard d(device);
        r = R.CommInitRank(&c, n_ranks, u, rank);  // rccl.h:220
    }
    if (r != ncclSuccess) {
        release(g.get(), false);
        return comm_fail("ncclCommInitRank", r);
    }
    g->m[0].comm = c;
    *out = g.release();
    return RTM_OK;
}

void rtm_group_destroy(rtm_group* g) {
    if (!g) return;
    // waits for the group's queued work, at most 600 s by default (far above any
    // queued sequence: 8192 frames at 7680x4320 drain in seconds), then aborts the
    // communicators, so a peer lost with a transfer unmatched cannot hang the caller
    // for ever.  A caller bounds it tighter with rtm_group_synchronize(g, timeout_ms)
    // first (the Python Group.close does); RTM_GROUP_DESTROY_TIMEOUT_MS sets the
    // bound (0: no limit)
    static const int32_t limit_ms = [] {
        const char* e = getenv("RTM_GROUP_DESTROY_TIMEOUT_MS");
        return e ? (int32_t)atoi(e) : 600000;
    }();
    if (!g->aborted) (void)rtm_group_synchronize(g, limit_ms);
    release(g, !g->aborted);
    delete g;
}

int rtm_group_info(rtm_group* g, int32_t* n_ranks, int32_t* n_local, int32_t* first_rank) {
    if (!g) return set_error(RTM_ERR_INVALID, "group is NULL");
    if (n_ranks) *n_ranks = g->n_ranks;
    if (n_local) *n_local = (int32_t)g->m.size();
    if (first_rank) *first_rank = g->m.empty() ? 0 : g->m[0].rank;
    return RTM_OK;
}

rtm_ctx* rtm_group_ctx(rtm_group* g, int32_t local) {
    if (!g || local < 0 || local >= (int32_t)g->m.size()) return nullptr;
    return g->m[(size_t)local].ctx;
}

int rtm_group_set_root_staging(rtm_group* g, int32_t on) {
    if (!g) return set_error(RTM_ERR_INVALID, "group is NULL");
    g->root_staging = on != 0;
    return RTM_OK;
}

namespace {

// A chunk of nf frames of the group (1 <= nf <= the staging slot's frame count),
// their inputs already validated and prepared.  Per member: the bands of all nf
// frames render on the member's context stream in one launch per pass (the batched
// kernels; the root's bands in place into out_dev[j], the others' into staging slot
// s, band j at offset j*band_bytes); the transfer stream waits for the render and
// then carries one gather per frame, so a context stream never waits for a
// transfer and the next chunk renders while this one is in flight.  Frame j is
// complete in the root's transfer-stream order (rtm_group_stream).
int group_stripe(const rtm_group* g) { return g->stripe >= 0 ? g->stripe : default_stripe(g->n_ranks); }

// The root's receive staging for striped RCCL gathers: one part per rank (its compact
// rows land here, then place_rows scatters them), on the root's device.
int ensure_recv(rtm_group* g, Member& rm, size_t bytes) {
    if (g->recv && bytes <= g->recv_bytes && g->recv_device == rm.device) return RTM_OK;
    // a bigger buffer, or the root moved to another device: the old buffer's last
    // receives and placements ran on the previous root's transfer stream
    for (Member& mb : g->m) {
        Guard d(mb.device);
        GHIP_TRY(hipStreamSynchronize(mb.xfer));
    }
    if (g->recv) {
        Guard d(g->recv_device);
        (void)hipFree(g->recv);
    }
    g->recv = nullptr;
    g->recv_bytes = 0;
    Guard d(rm.device);
    if (hipMalloc(&g->recv, bytes) != hipSuccess) return set_error(RTM_ERR_OOM, "receive staging allocation failed");
    g->recv_bytes = bytes;
    g->recv_device = rm.device;
    return RTM_OK;
}

// lanes[i]: the lane of member i that renders this chunk (its context's streams,
// rtm::internal::lanes_begin)
int group_chunk(rtm_group* g, const rtm::internal::PreparedFrame* const* pf, int nf, int32_t width, int32_t height,
                int32_t format, int32_t root, void* const* out_dev, const int* lanes) {
    const int32_t n = g->n_ranks;
    const int32_t S = group_stripe(g);
    const size_t row_bytes = (size_t)rtm::internal::bytes_per_pixel(format) * (size_t)width;
    const size_t part_bytes = row_bytes * (size_t)part_of(height, n, S, 0).rows;  // rank 0 holds the most rows
    int rc;
    std::vector<void*> outs((size_t)nf);
    // 1. every local member renders its rows of the chunk's frames
    for (size_t mi = 0; mi < g->m.size(); ++mi) {
        Member& mb = g->m[mi];
        Part pt = part_of(height, n, S, mb.rank);
        Guard d(mb.device);
        hipStream_t rs = rtm::internal::lane_stream(mb.ctx, lanes[mi]);
        const bool staged = mb.rank != root || g->root_staging;
        if (pt.rows > 0) {
            const int sl = mb.slot;
            if (staged) GHIP_TRY(hipStreamWaitEvent(rs, mb.sent[sl], 0));  // slot sl's previous sends have read it
            const bool stripes = pt.map.stripe_rows > 0;
            // the root in place: its stripes straight at their image rows (out_global)
            pt.map.out_global = (!staged && stripes) ? 1 : 0;
            for (int j = 0; j < nf; ++j)
                outs[(size_t)j] = staged ? (void*)((char*)mb.stage[sl] + part_bytes * (size_t)j)
                                         : stripes ? out_dev[j]
                                                   : (void*)((char*)out_dev[j] + row_bytes * (size_t)pt.r0);
            rc = stripes ? rtm::internal::enqueue_prepared_batch(mb.ctx, pf, nf, format, 0, pt.rows, outs.data(),
                                                                 &pt.map, lanes[mi])
                         : rtm::internal::enqueue_prepared_batch(mb.ctx, pf, nf, format, pt.r0, pt.r0 + pt.rows,
                                                                 outs.data(), nullptr, lanes[mi]);
            if (rc) return rc;
            if (staged) {
                GHIP_TRY(hipEventRecord(mb.ready[sl], rs));
                GHIP_TRY(hipStreamWaitEvent(mb.xfer, mb.ready[sl], 0));
            }
        }
        if (mb.rank == root && !staged) {  // the root's own rows, in the frames' completion order
            GHIP_TRY(hipEventRecord(mb.start, rs));
            GHIP_TRY(hipStreamWaitEvent(mb.xfer, mb.start, 0));
        }
    }
    // 2. ONE gather per frame: the root receives every other part, the others send
    //    theirs (nothing to move for a one-rank group rendering in place).  A part lands
    //    in place (a contiguous band) or compact in the root's receive staging (stripes),
    //    and after the frame's transfers the root places the staged parts at their image
    //    rows.  The transfers are RCCL's matched sends and receives, or with the loopback
    //    transport device copies of the same bytes to the same places, in RCCL's
    //    completion order for a pair (the copy runs once the sender's transfer stream
    //    reached its send; the sender's stream moves past its send once the copy read it).
    Member* rm = nullptr;
    for (Member& mb : g->m)
        if (mb.rank == root) rm = &mb;
    if (n > 1 || g->root_staging) {
        const Rccl& R = rccl();
        const bool stripes = S > 0 && n > 1;
        if (stripes && rm && (rc = ensure_recv(g, *rm, part_bytes * (size_t)n))) return rc;
        auto dst_of = [&](int j, int32_t p) -> void* {
            return stripes ? (void*)((char*)g->recv + part_bytes * (size_t)p)
                           : (void*)((char*)out_dev[j] + row_bytes * (size_t)part_of(height, n, S, p).r0);
        };
        for (int j = 0; j < nf; ++j) {
            if (g->loopback) {
                for (Member& mb : g->m) {
                    const bool staged = mb.rank != root || g->root_staging;
                    const Part pt = part_of(height, n, S, mb.rank);
                    if (!staged || pt.rows <= 0) continue;
                    GHIP_TRY(hipEventRecord(mb.lb_sent, mb.xfer));
                    GHIP_TRY(hipStreamWaitEvent(rm->xfer, mb.lb_sent, 0));
                    GHIP_TRY(hipMemcpyAsync(dst_of(j, mb.rank), (char*)mb.stage[mb.slot] + part_bytes * (size_t)j,
                                            row_bytes * (size_t)pt.rows, hipMemcpyDeviceToDevice, rm->xfer));
                    GHIP_TRY(hipEventRecord(mb.lb_recv, rm->xfer));
                    GHIP_TRY(hipStreamWaitEvent(mb.xfer, mb.lb_recv, 0));
                }
            } else {
                NCCL_TRY(R.GroupStart());
                for (Member& mb : g->m) {
                    if (mb.rank == root) {
                        for (int32_t p = 0; p < n; ++p) {
                            if (p == root && !g->root_staging) continue;
                            const Part pt = part_of(height, n, S, p);
                            if (pt.rows <= 0) continue;
                            ncclResult_t r = R.Recv(dst_of(j, p), row_bytes * (size_t)pt.rows, ncclUint8, p, mb.comm,
                                                    mb.xfer);
                            if (r != ncclSuccess) {
                                (void)R.GroupEnd();
                                return comm_fail("ncclRecv", r);
                            }
                        }
                    }
                    const Part pt = part_of(height, n, S, mb.rank);
                    const bool staged = mb.rank != root || g->root_staging;
                    if (staged && pt.rows > 0) {
                        ncclResult_t r = R.Send((char*)mb.stage[mb.slot] + part_bytes * (size_t)j,
                                                row_bytes * (size_t)pt.rows, ncclUint8, root, mb.comm, mb.xfer);
                        if (r != ncclSuccess) {
                            (void)R.GroupEnd();
                            return comm_fail("ncclSend", r);
                        }
                    }
                }
                NCCL_TRY(R.GroupEnd());
            }
            if (stripes && rm) {  // the received parts to their image rows, in the root's transfer order
                Guard d(rm->device);
                for (int32_t p = 0; p < n; ++p) {
                    if (p == root && !g->root_staging) continue;
                    GHIP_TRY(place_rows(out_dev[j], (char*)g->recv + part_bytes * (size_t)p, part_of(height, n, S, p),
                                        row_bytes, hipMemcpyDeviceToDevice, rm->xfer));
                }
            }
        }
    }
    // 3. staging slots: free again once their sends have read them
    for (Member& mb : g->m) {
        const Part pt = part_of(height, n, S, mb.rank);
        const bool staged = mb.rank != root || g->root_staging;
        if (staged && pt.rows > 0) {
            Guard d(mb.device);
            GHIP_TRY(hipEventRecord(mb.sent[mb.slot], mb.xfer));
            mb.slot = (mb.slot + 1) % mb.nstage;
        }
    }
    return RTM_OK;
}

struct PreparedDeleter {
    void operator()(rtm::internal::PreparedFrame* f) const { rtm::internal::delete_prepared(f); }
};

// Shared checks of the frame calls; allocates the staging buffers (slots[mi] slots of
// `frames` parts each on local member mi; nullptr: one slot).
int group_begin(rtm_group* g, int32_t width, int32_t height, int32_t format, int32_t root, int32_t frames,
                const int* slots = nullptr) {
    if (!g) return set_error(RTM_ERR_INVALID, "group is NULL");
    if (g->aborted) return set_error(RTM_ERR_COMM, "group was aborted");
    if (root < 0 || root >= g->n_ranks) return set_error(RTM_ERR_INVALID, "root outside [0, n_ranks)");
    const int32_t bpp = rtm::internal::bytes_per_pixel(format);
    if (!bpp) return set_error(RTM_ERR_INVALID, "unknown output format");
    if (width <= 0 || height <= 0 || width > RTM_MAX_DIM || height > RTM_MAX_DIM)
        return set_error(RTM_ERR_INVALID, "image size outside [1, RTM_MAX_DIM]");
    const int32_t rows0 = part_of(height, g->n_ranks, group_stripe(g), 0).rows;  // the largest part
    for (size_t mi = 0; mi < g->m.size(); ++mi) {
        Member& mb = g->m[mi];
        const bool staged = mb.rank != root || g->root_staging;
        int rc;
        if (staged && (rc = ensure_stage(mb, (size_t)bpp * (size_t)width * (size_t)rows0 * (size_t)frames,
                                         slots ? slots[mi] : 1)))
            return rc;
    }
    return RTM_OK;
}

// Does any frame of one chunk overlap a frame of another chunk on a different lane
// (chunk c on lane c % L)?  Such frames would be written side by side, so the later
// frame might not land last.  Frames of equal size: sorting by address, any two
// overlapping ones are joined by a chain of overlapping neighbours, so checking
// sorted neighbours checks every pair (rtm_api.cpp frame_lanes).
bool chunks_clash_across_lanes(const std::vector<std::pair<int32_t, int32_t>>& chunks, void* const* out_dev,
                               uintptr_t frame_bytes, int L) {
    if (L <= 1) return false;
    std::vector<std::pair<uintptr_t, int>> r;
    for (size_t c = 0; c < chunks.size(); ++c)
        for (int32_t k = 0; k < chunks[c].second; ++k)
            r.push_back({(uintptr_t)out_dev[chunks[c].first + k], (int)(c % (size_t)L)});
    std::sort(r.begin(), r.end());
    for (size_t i = 1; i < r.size(); ++i)
        if (r[i].first < r[i - 1].first + frame_bytes && r[i].second != r[i - 1].second) return true;
    return false;
}

int check_root_out(rtm_group* g, int32_t format, int32_t root, void* out) {
    for (const Member& mb : g->m)
        if (mb.rank == root) {
            if (!out) return set_error(RTM_ERR_INVALID, "out_dev is NULL on the root");
            if (format == RTM_FORMAT_RGBA32F && ((uintptr_t)out & 15))
                return set_error(RTM_ERR_INVALID, "RGBA32F output must be 16-byte aligned");
        }
    return RTM_OK;
}

}  // namespace

int rtm_group_render_async(rtm_group* g, const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow,
                           int32_t width, int32_t height, int32_t march_steps, int32_t flags, int32_t format,
                           int32_t root, void* out_dev) {
    void* outs[1] = {out_dev};
    return rtm_group_render_frames_async(g, 1, scene, eye, shadow, width, height, march_steps, flags, format, root,
                                         outs);
}

int rtm_group_render_frames_async(rtm_group* g, int32_t n_frames, const rtm_scene* scenes, const rtm_camera* eye,
                                  const rtm_camera* shadow, int32_t width, int32_t height, int32_t march_steps,
                                  int32_t flags, int32_t format, int32_t root, void* const* out_dev) {
    if (!g) return set_error(RTM_ERR_INVALID, "group is NULL");
    if (n_frames < 1 || !scenes || !out_dev) return set_error(RTM_ERR_INVALID, "bad frame list");
    if (width <= 0 || height <= 0 || width > RTM_MAX_DIM || height > RTM_MAX_DIM)
        return set_error(RTM_ERR_INVALID, "image size outside [1, RTM_MAX_DIM]");
    // frames per launch: the library's auto rule for a band (every rank's bands of a
    // chunk render in one launch per pass), the same on every rank
    const int32_t rows0 = part_of(height, g->n_ranks > 0 ? g->n_ranks : 1, group_stripe(g), 0).rows;
    const int32_t B = std::max(1, std::min<int32_t>(n_frames, rtm::internal::auto_frames_per_launch(width, rows0)));
    if (root < 0 || root >= g->n_ranks) return set_error(RTM_ERR_INVALID, "root outside [0, n_ranks)");
    const int32_t bpp = rtm::internal::bytes_per_pixel(format);
    if (!bpp) return set_error(RTM_ERR_INVALID, "unknown output format");
    bool holds_root = false;
    for (const Member& mb : g->m) holds_root |= mb.rank == root;
    const uintptr_t frame_bytes = (uintptr_t)bpp * (uintptr_t)width * height;
    // The chunks: B frames each, except that on the root a chunk's frames need disjoint
    // outputs (they render side by side), so a repeated output starts the next chunk
    // and the later frame still lands last (chunking is local: every frame's gather is
    // its own matched send/receive set).
    std::vector<std::pair<int32_t, int32_t>> chunks;  // (first frame, frames)
    for (int32_t i0 = 0; i0 < n_frames;) {
        int nf = std::min<int32_t>(B, n_frames - i0);
        if (holds_root)
            for (int k = 1; k < nf; ++k) {
                bool clash = false;
                for (int q = 0; q < k && !clash; ++q) {
                    const uintptr_t a = (uintptr_t)out_dev[i0 + k], b = (uintptr_t)out_dev[i0 + q];
                    clash = a < b + frame_bytes && b < a + frame_bytes;
                }
                if (clash) {
                    nf = k;
                    break;
                }
            }
        chunks.push_back({i0, nf});
        i0 += nf;
    }
    const int32_t n_chunks = (int32_t)chunks.size();
    // Every member spreads the chunks over its context's lanes, as rtm_render_frames_async
    // spreads batches (chunk c on lane c % L).  A member rendering the root's rows in place
    // writes the caller's frames from its lanes: where frames of chunks on different lanes
    // overlap (one buffer reused across chunks) it keeps one lane, so they land in order.
    std::vector<int> L(g->m.size(), 1), lane(g->m.size(), 0), cap(g->m.size(), 0), slots(g->m.size(), 1);
    for (size_t mi = 0; mi < g->m.size(); ++mi) {
        const Member& mb = g->m[mi];
        const int32_t rows = part_of(height, g->n_ranks, group_stripe(g), mb.rank).rows;
        if (rows <= 0) continue;
        const int l = rtm::internal::lanes_plan(mb.ctx, width, rows, n_chunks);
        const bool in_place = mb.rank == root && !g->root_staging;
        cap[mi] = in_place && chunks_clash_across_lanes(chunks, out_dev, frame_bytes, l) ? 1 : 0;
        slots[mi] = std::min(NSLOT, (cap[mi] ? 1 : l) + 1);
    }
    int rc = group_begin(g, width, height, format, root, B, slots.data());
    if (rc) return rc;
    // more than one band: each evaluates the shadow texels it reads (same image bits)
    const int32_t f = flags | (g->n_ranks > 1 ? RTM_FLAG_FUSED_SHADOW : 0);
    // Everything that can fail for the caller's inputs is checked before the first
    // enqueue: a rank that stopped half-way would leave its peers' transfers unmatched.
    for (int32_t i = 0; i < n_frames; ++i) {
        if ((rc = rtm::internal::check_frame(&scenes[i], eye, shadow, width, height, march_steps, f))) return rc;
        if ((rc = check_root_out(g, format, root, out_dev[i]))) return rc;
    }
    std::vector<std::unique_ptr<rtm::internal::PreparedFrame, PreparedDeleter>> pf((size_t)B);
    std::vector<const rtm::internal::PreparedFrame*> pp((size_t)B);
    for (int32_t k = 0; k < B; ++k) {
        pf[(size_t)k].reset(rtm::internal::new_prepared());
        if (!pf[(size_t)k]) return set_error(RTM_ERR_OOM, "host allocation failed");
        pp[(size_t)k] = pf[(size_t)k].get();
    }
    // the lanes join the context stream at the end (rtm_group_synchronize waits on it)
    for (size_t mi = 0; mi < g->m.size(); ++mi) {
        const int32_t rows = part_of(height, g->n_ranks, group_stripe(g), g->m[mi].rank).rows;
        if (rows <= 0) continue;
        Guard d(g->m[mi].device);
        const int l = rtm::internal::lanes_begin(g->m[mi].ctx, width, rows, n_chunks, cap[mi]);
        if (l < 0) {
            for (size_t q = 0; q < mi; ++q) (void)rtm::internal::lanes_end(g->m[q].ctx, L[q]);
            return l;
        }
        L[mi] = l;
    }
    auto join = [&]() {
        int jr = RTM_OK;
        for (size_t mi = 0; mi < g->m.size(); ++mi) {
            Guard d(g->m[mi].device);
            const int r = rtm::internal::lanes_end(g->m[mi].ctx, L[mi]);
            if (r && !jr) jr = r;
        }
        return jr;
    };
    for (int32_t c = 0; c < n_chunks; ++c) {
        const int32_t i0 = chunks[(size_t)c].first, nf = chunks[(size_t)c].second;
        for (int k = 0; k < nf && !rc; ++k)
            rc = rtm::internal::prepare_frame(pf[(size_t)k].get(), &scenes[i0 + k], eye, shadow, width, height,
                                              march_steps, f);
        for (size_t mi = 0; mi < g->m.size(); ++mi) lane[mi] = c % L[mi];
        if (!rc) rc = group_chunk(g, pp.data(), nf, width, height, format, root, out_dev + i0, lane.data());
        if (rc) {
            (void)join();  // the context streams still cover what was enqueued
            return rc;
        }
    }
    return join();
}

namespace {

// rtm_group_render with host_direct: every member renders its band into its own
// staging buffer and copies it from its device straight into its rows of out_host
// (one host thread per member: a pageable copy blocks its caller, and into a
// registered buffer each copy is DMA over that device's own PCIe link) -- N links
// into host memory instead of a gather into one device and that device's link.
int group_render_direct(rtm_group* g, const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow,
                        int32_t width, int32_t height, int32_t march_steps, int32_t flags, int32_t format,
                        void* out_host) {
    if ((int32_t)g->m.size() != g->n_ranks)
        return set_error(RTM_ERR_UNSUPPORTED, "direct host delivery needs every rank in this process");
    if (!out_host) return set_error(RTM_ERR_INVALID, "out_host is NULL");
    int rc = rtm_group_synchronize(g, 0);  // staging buffers idle
    if (rc) return rc;
    const int32_t n = g->n_ranks;
    const size_t row_bytes = (size_t)rtm::internal::bytes_per_pixel(format) * (size_t)width;
    const int32_t f = flags | (n > 1 ? RTM_FLAG_FUSED_SHADOW : 0);
    if ((rc = rtm::internal::check_frame(scene, eye, shadow, width, height, march_steps, f))) return rc;
    const int32_t S = group_stripe(g);
    for (Member& mb : g->m)
        if ((rc = ensure_stage(mb, row_bytes * (size_t)part_of(height, n, S, 0).rows, 1))) return rc;
    std::unique_ptr<rtm::internal::PreparedFrame, PreparedDeleter> pf(rtm::internal::new_prepared());
    if (!pf) return set_error(RTM_ERR_OOM, "host allocation failed");
    if ((rc = rtm::internal::prepare_frame(pf.get(), scene, eye, shadow, width, height, march_steps, f))) return rc;
    for (Member& mb : g->m) {
        const Part pt = part_of(height, n, S, mb.rank);
        if (pt.rows <= 0) continue;
        Guard d(mb.device);
        rc = pt.map.stripe_rows > 0
                 ? rtm::internal::enqueue_prepared(mb.ctx, pf.get(), format, 0, pt.rows, mb.stage[0], &pt.map)
                 : rtm::internal::enqueue_prepared(mb.ctx, pf.get(), format, pt.r0, pt.r0 + pt.rows, mb.stage[0]);
        if (rc) return rc;
    }
    std::vector<int> rcs(g->m.size(), RTM_OK);
    std::vector<std::string> errs(g->m.size());
    auto copy_part = [&](size_t i) {
        Member& mb = g->m[i];
        Guard d(mb.device);
        hipStream_t rs = rtm::internal::ctx_stream(mb.ctx);
        hipError_t e = place_rows(out_host, mb.stage[0], part_of(height, n, S, mb.rank), row_bytes,
                                  hipMemcpyDeviceToHost, rs);
        if (e == hipSuccess) e = hipStreamSynchronize(rs);
        if (e != hipSuccess) {
            rcs[i] = RTM_ERR_HIP;
            errs[i] = std::string("band copy from device ") + std::to_string(mb.device) + ": " + hipGetErrorString(e);
        }
    };
    std::vector<size_t> live;
    for (size_t i = 0; i < g->m.size(); ++i)
        if (part_of(height, n, S, g->m[i].rank).rows > 0) live.push_back(i);
    if (live.size() <= 1) {
        for (size_t i : live) copy_part(i);
    } else {
        std::vector<std::thread> th;
        for (size_t i : live) th.emplace_back(copy_part, i);
        for (auto& t : th) t.join();
    }
    for (size_t i = 0; i < g->m.size(); ++i)
        if (rcs[i]) return set_error(rcs[i], errs[i].c_str());
    return RTM_OK;
}

}  // namespace

int rtm_group_set_partition(rtm_group* g, int32_t stripe_rows) {
    if (!g) return set_error(RTM_ERR_INVALID, "group is NULL");
    if (stripe_rows < -1 || stripe_rows > RTM_MAX_DIM) return set_error(RTM_ERR_INVALID, "stripe_rows outside [-1, RTM_MAX_DIM]");
    if ((int64_t)stripe_rows * g->n_ranks > (int64_t)RTM_MAX_DIM * 8)  // the stripe period stays an int32 row count
        return set_error(RTM_ERR_INVALID, "stripe period stripe_rows * n_ranks too large");
    const int rc = rtm_group_synchronize(g, 0);  // frames in flight keep the partition they were issued with
    if (rc) return rc;
    g->stripe = stripe_rows;
    return RTM_OK;
}

int32_t rtm_group_partition(rtm_group* g) { return g ? group_stripe(g) : -1; }

int rtm_group_frames_plan(rtm_group* g, int32_t width, int32_t height, int32_t n_frames, int32_t root,
                          int32_t* frames_per_chunk, int32_t* lanes) {
    if (!g || !frames_per_chunk || !lanes || width < 1 || height < 1 || n_frames < 1 || root < 0 ||
        root >= g->n_ranks || g->m.empty())
        return set_error(RTM_ERR_INVALID, "bad arguments");
    // rtm_group_render_frames_async's rules: chunks of the auto frames per launch of part
    // 0, and each member's lanes_plan over the chunks (distinct outputs: no clash cap)
    const int32_t rows0 = part_of(height, g->n_ranks, group_stripe(g), 0).rows;
    const int32_t B = std::max(1, std::min<int32_t>(n_frames, rtm::internal::auto_frames_per_launch(width, rows0)));
    const Member* mb = &g->m[0];
    for (const Member& m : g->m)
        if (m.rank == root) mb = &m;
    const int32_t rows = part_of(height, g->n_ranks, group_stripe(g), mb->rank).rows;
    *frames_per_chunk = B;
    *lanes = rows > 0 ? rtm::internal::lanes_plan(mb->ctx, width, rows, (n_frames + B - 1) / B) : 1;
    return RTM_OK;
}

int rtm_group_set_host_direct(rtm_group* g, int32_t on) {
    if (!g) return set_error(RTM_ERR_INVALID, "group is NULL");
    if (on && (int32_t)g->m.size() != g->n_ranks)
        return set_error(RTM_ERR_UNSUPPORTED, "direct host delivery needs every rank in this process");
    g->host_direct = on != 0;
    return RTM_OK;
}

int rtm_group_render(rtm_group* g, const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow,
                     int32_t width, int32_t height, int32_t march_steps, int32_t flags, int32_t format,
                     void* out_host) {
    if (!g) return set_error(RTM_ERR_INVALID, "group is NULL");
    if (g->aborted) return set_error(RTM_ERR_COMM, "group was aborted");
    const int32_t bpp = rtm::internal::bytes_per_pixel(format);
    if (!bpp) return set_error(RTM_ERR_INVALID, "unknown output format");
    if (width <= 0 || height <= 0 || width > RTM_MAX_DIM || height > RTM_MAX_DIM)
        return set_error(RTM_ERR_INVALID, "image size outside [1, RTM_MAX_DIM]");
    if (g->host_direct) return group_render_direct(g, scene, eye, shadow, width, height, march_steps, flags, format,
                                                   out_host);
    Member* root = nullptr;
    for (Member& mb : g->m)
        if (mb.rank == 0) root = &mb;
    const size_t bytes = (size_t)bpp * (size_t)width * (size_t)height;
    if (root) {
        if (!out_host) return set_error(RTM_ERR_INVALID, "out_host is NULL on the root");
        if (g->root_frame_bytes < bytes) {
            Guard d(root->device);
            GHIP_TRY(hipStreamSynchronize(root->xfer));
            if (g->root_frame) (void)hipFree(g->root_frame);
            g->root_frame = nullptr;
            g->root_frame_bytes = 0;
            if (hipMalloc(&g->root_frame, bytes) != hipSuccess)
                return set_error(RTM_ERR_OOM, "root frame allocation failed");
            g->root_frame_bytes = bytes;
        }
    }
    void* outs[1] = {root ? g->root_frame : nullptr};
    int rc = rtm_group_render_frames_async(g, 1, scene, eye, shadow, width, height, march_steps, flags, format, 0,
                                           outs);
    if (rc) return rc;
    if (root) {  // the frame is complete in the root's transfer-stream order
        Guard d(root->device);
        GHIP_TRY(hipMemcpyAsync(out_host, g->root_frame, bytes, hipMemcpyDeviceToHost, root->xfer));
        // wait in the runtime (a pageable copy is staged by the waiting thread: polling
        // the stream instead took 23 ms per 4K frame instead of 2.4)
        GHIP_TRY(hipStreamSynchronize(root->xfer));
    }
    return rtm_group_synchronize(g, 0);
}

void* rtm_group_stream(rtm_group* g) {
    if (!g || g->m.empty()) return nullptr;
    for (const Member& mb : g->m)
        if (mb.rank == 0) return (void*)mb.xfer;
    return (void*)g->m[0].xfer;
}

int rtm_group_synchronize(rtm_group* g, int32_t timeout_ms) {
    if (!g) return set_error(RTM_ERR_INVALID, "group is NULL");
    if (g->aborted) return set_error(RTM_ERR_COMM, "group was aborted");
    const Rccl& R = rccl();
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        bool busy = false;
        for (Member& mb : g->m) {
            Guard d(mb.device);
            for (hipStream_t s : {rtm::internal::ctx_stream(mb.ctx), mb.xfer}) {
                const hipError_t e = hipStreamQuery(s);
                if (e == hipErrorNotReady) busy = true;
                else if (e != hipSuccess) return hip_fail("hipStreamQuery", e);
            }
            ncclResult_t ae = ncclSuccess;
            if (mb.comm && R.CommGetAsyncError && R.CommGetAsyncError(mb.comm, &ae) == ncclSuccess &&
                ae != ncclSuccess && ae != ncclInProgress) {
                for (Member& m2 : g->m)
                    if (m2.comm) (void)R.CommAbort(m2.comm);
                for (Member& m2 : g->m) m2.comm = nullptr;
                g->aborted = true;
                return comm_fail("RCCL asynchronous error (communicators aborted)", ae);
            }
        }
        if (!busy) return RTM_OK;
        if (timeout_ms > 0 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) {
            for (Member& mb : g->m)
                if (mb.comm) (void)R.CommAbort(mb.comm);
            for (Member& mb : g->m) mb.comm = nullptr;
            g->aborted = true;
            return set_error(RTM_ERR_COMM, "group work did not finish in time (communicators aborted)");
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

}  // extern "C"
