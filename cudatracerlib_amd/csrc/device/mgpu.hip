// mgpu.hip — multi-GPU half of the C ABI: the PixelData reduce of a tile-sharded
// render over RCCL (include/ctl_trace.h "multi-GPU").
//
// The path shards by image tiles with no exchange during rendering; the one
// collective is a sum-reduce of the per-rank framebuffers (7 floats per
// pixel) to the root.  Over xGMI (point-to-point links, ring reduce) that is
// 58 MB at 1080p.  The reduce reads the rank framebuffers and writes the sum
// into a separate buffer on the root: the rank framebuffers keep accumulating
// their own pixels only, so the reduce may run after any step, any number of
// times (an in-place reduce would fold the other ranks' totals into the
// root's accumulator and count them again at the next reduce).
//
// RCCL is loaded on first use (dlopen), so single-GPU and host-only users of
// libctl_trace.so do not need it at load time.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"

namespace {

// The RCCL entry points this file calls, resolved from librccl on first use.
struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclReduce) reduce = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclCommUserRank) user_rank = nullptr;   // required: tells a rank whether it is the root
    std::string err;
    bool ok = false;
};

const Rccl& rccl() {
    static Rccl R;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) { R.err = std::string("RCCL not loadable: ") + dlerror(); return; }
        bool all = true;
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn) all = false;
        };
        sym(R.get_unique_id, "ncclGetUniqueId");
        sym(R.comm_init_rank, "ncclCommInitRank");
        sym(R.comm_init_all, "ncclCommInitAll");
        sym(R.comm_destroy, "ncclCommDestroy");
        sym(R.reduce, "ncclReduce");
        sym(R.group_start, "ncclGroupStart");
        sym(R.group_end, "ncclGroupEnd");
        sym(R.error_string, "ncclGetErrorString");
        // every rank of a collective must be able to tell whether a NULL d_out
        // would reach RCCL as the root's receive buffer (ctl_fb_reduce): without
        // ncclCommUserRank all ranks refuse alike (CTL_ERR_NODEVICE), none waits
        sym(R.user_rank, "ncclCommUserRank");
        if (!all) { R.err = "RCCL: missing entry points"; return; }
        R.ok = true;
    });
    return R;
}

ctl_status nccl_status(ctl_ctx* c, ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return CTL_OK;
    if (c) c->err = std::string(what) + ": " + rccl().error_string(r);
    return r == ncclInvalidArgument || r == ncclInvalidUsage ? CTL_ERR_INVALID : CTL_ERR_HIP;
}

bool have_rccl(ctl_ctx* c) {
    if (rccl().ok) return true;
    if (c) c->err = rccl().err;
    return false;
}

}  // namespace

extern "C" {

CTL_API ctl_status ctl_comm_unique_id(void* id_out) {
    if (!id_out) return CTL_ERR_INVALID;
    static_assert(sizeof(ncclUniqueId) == CTL_COMM_ID_BYTES, "ncclUniqueId is 128 bytes");
    if (!have_rccl(nullptr)) return CTL_ERR_NODEVICE;
    ncclUniqueId id;
    if (rccl().get_unique_id(&id) != ncclSuccess) return CTL_ERR_HIP;
    std::memcpy(id_out, &id, sizeof(id));
    return CTL_OK;
}

CTL_API ctl_status ctl_comm_init_rank(void** comm_out, int32_t nranks, const void* id, int32_t rank, int32_t device) {
    if (!comm_out || !id || nranks < 1 || rank < 0 || rank >= nranks) return CTL_ERR_INVALID;
    if (!have_rccl(nullptr)) return CTL_ERR_NODEVICE;
    if (hipSetDevice(device) != hipSuccess) return CTL_ERR_NODEVICE;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm = nullptr;
    if (rccl().comm_init_rank(&comm, nranks, uid, rank) != ncclSuccess) return CTL_ERR_HIP;
    *comm_out = comm;
    return CTL_OK;
}

CTL_API ctl_status ctl_comm_init_all(void** comms_out, int32_t ndev, const int32_t* devices) {
    if (!comms_out || ndev < 1) return CTL_ERR_INVALID;
    if (!have_rccl(nullptr)) return CTL_ERR_NODEVICE;
    std::vector<ncclComm_t> comms((size_t)ndev, nullptr);
    std::vector<int> devs((size_t)ndev);
    for (int i = 0; i < ndev; i++) devs[(size_t)i] = devices ? devices[i] : i;
    if (rccl().comm_init_all(comms.data(), ndev, devs.data()) != ncclSuccess) return CTL_ERR_HIP;
    for (int i = 0; i < ndev; i++) comms_out[i] = comms[(size_t)i];
    return CTL_OK;
}

CTL_API ctl_status ctl_comm_destroy(void* comm) {
    if (!comm) return CTL_ERR_INVALID;
    if (!have_rccl(nullptr)) return CTL_ERR_NODEVICE;
    return rccl().comm_destroy(reinterpret_cast<ncclComm_t>(comm)) == ncclSuccess ? CTL_OK : CTL_ERR_HIP;
}

CTL_API ctl_status ctl_fb_reduce(ctl_ctx* c, void* comm, const ctl_pixel* d_fb, ctl_pixel* d_out, uint64_t n_pixels,
                                 int32_t root, void* stream) {
    if (!c || !comm || (!d_fb && n_pixels)) return CTL_ERR_INVALID;
    if (d_out && d_out == d_fb) { c->err = "fb_reduce: d_out must not alias d_fb"; return CTL_ERR_INVALID; }
    if (!have_rccl(c)) return CTL_ERR_NODEVICE;
    if (!d_out && n_pixels) {
        // the root needs a receive buffer: a NULL d_out never reaches RCCL as the
        // root's recvbuff.  A non-root rank may pass NULL.  A rank whose number
        // cannot be read refuses too (its peers then fail in the collective rather
        // than the root writing through a null pointer).
        int me = -1;
        if (rccl().user_rank(reinterpret_cast<ncclComm_t>(comm), &me) != ncclSuccess) {
            c->err = "fb_reduce: the rank cannot be read (ncclCommUserRank) and d_out is NULL";
            return CTL_ERR_INVALID;
        }
        if (me == root) {
            c->err = "fb_reduce: d_out is required on the root rank";
            return CTL_ERR_INVALID;
        }
    }
    if (hipSetDevice(c->device) != hipSuccess) { c->err = "fb_reduce: hipSetDevice failed"; return CTL_ERR_HIP; }
    const size_t count = (size_t)n_pixels * (sizeof(ctl_pixel) / sizeof(float));
    return nccl_status(c, rccl().reduce(d_fb, d_out, count, ncclFloat, ncclSum, root,
                                        reinterpret_cast<ncclComm_t>(comm), reinterpret_cast<hipStream_t>(stream)),
                       "fb_reduce: ncclReduce");
}

CTL_API ctl_status ctl_fb_reduce_all(ctl_ctx* const* ctxs, void* const* comms, const ctl_pixel* const* d_fbs,
                                     ctl_pixel* d_out, int32_t n, uint64_t n_pixels, int32_t root,
                                     void* const* streams) {
    if (!ctxs || !comms || !d_fbs || n < 1 || root < 0 || root >= n) return CTL_ERR_INVALID;
    if (!have_rccl(ctxs[0])) return CTL_ERR_NODEVICE;
    if (!d_out && n_pixels) { ctxs[0]->err = "fb_reduce_all: d_out (on the root's GPU) is required"; return CTL_ERR_INVALID; }
    if (d_out && d_out == d_fbs[root]) { ctxs[0]->err = "fb_reduce_all: d_out must not alias d_fbs[root]"; return CTL_ERR_INVALID; }
    const size_t count = (size_t)n_pixels * (sizeof(ctl_pixel) / sizeof(float));
    if (rccl().group_start() != ncclSuccess) return CTL_ERR_HIP;
    ctl_status st = CTL_OK;
    for (int i = 0; i < n && st == CTL_OK; i++) {
        ctl_ctx* c = ctxs[i];
        if (!c || !comms[i]) { st = CTL_ERR_INVALID; break; }
        if (hipSetDevice(c->device) != hipSuccess) { c->err = "fb_reduce_all: hipSetDevice failed"; st = CTL_ERR_HIP; break; }
        st = nccl_status(c, rccl().reduce(d_fbs[i], i == root ? d_out : nullptr, count, ncclFloat, ncclSum, root,
                                          reinterpret_cast<ncclComm_t>(comms[i]),
                                          reinterpret_cast<hipStream_t>(streams ? streams[i] : nullptr)),
                         "fb_reduce_all: ncclReduce");
    }
    const ncclResult_t g = rccl().group_end();
    if (st != CTL_OK) return st;
    return nccl_status(ctxs[0], g, "fb_reduce_all: ncclGroupEnd");
}

}  // extern "C"
