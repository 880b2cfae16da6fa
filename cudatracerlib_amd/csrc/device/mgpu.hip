// mgpu.hip — multi-GPU half of the C ABI: the PixelData reduce of a tile-sharded
// render over RCCL (include/ctl_trace.h "multi-GPU").
//
// The path shards by image tiles with no exchange during rendering; the one
// collective is a sum-reduce of the per-rank framebuffers (7 floats per
// pixel) to the root, once per progressive step or at the end.  Over xGMI
// (point-to-point links, ring reduce) that is 58 MB at 1080p; ncclReduce moves
// it once per link, in place on every rank.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

#include "common.h"

namespace {

ctl_status nccl_status(ctl_ctx* c, ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return CTL_OK;
    if (c) c->err = std::string(what) + ": " + ncclGetErrorString(r);
    return r == ncclInvalidArgument || r == ncclInvalidUsage ? CTL_ERR_INVALID : CTL_ERR_HIP;
}

}  // namespace

extern "C" {

CTL_API ctl_status ctl_comm_unique_id(void* id_out) {
    if (!id_out) return CTL_ERR_INVALID;
    static_assert(sizeof(ncclUniqueId) == CTL_COMM_ID_BYTES, "ncclUniqueId is 128 bytes");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return CTL_ERR_HIP;
    std::memcpy(id_out, &id, sizeof(id));
    return CTL_OK;
}

CTL_API ctl_status ctl_comm_init_rank(void** comm_out, int32_t nranks, const void* id, int32_t rank, int32_t device) {
    if (!comm_out || !id || nranks < 1 || rank < 0 || rank >= nranks) return CTL_ERR_INVALID;
    if (hipSetDevice(device) != hipSuccess) return CTL_ERR_NODEVICE;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm = nullptr;
    if (ncclCommInitRank(&comm, nranks, uid, rank) != ncclSuccess) return CTL_ERR_HIP;
    *comm_out = comm;
    return CTL_OK;
}

CTL_API ctl_status ctl_comm_init_all(void** comms_out, int32_t ndev, const int32_t* devices) {
    if (!comms_out || ndev < 1) return CTL_ERR_INVALID;
    std::vector<ncclComm_t> comms((size_t)ndev, nullptr);
    std::vector<int> devs((size_t)ndev);
    for (int i = 0; i < ndev; i++) devs[(size_t)i] = devices ? devices[i] : i;
    if (ncclCommInitAll(comms.data(), ndev, devs.data()) != ncclSuccess) return CTL_ERR_HIP;
    for (int i = 0; i < ndev; i++) comms_out[i] = comms[(size_t)i];
    return CTL_OK;
}

CTL_API ctl_status ctl_comm_destroy(void* comm) {
    if (!comm) return CTL_ERR_INVALID;
    return ncclCommDestroy(reinterpret_cast<ncclComm_t>(comm)) == ncclSuccess ? CTL_OK : CTL_ERR_HIP;
}

CTL_API ctl_status ctl_fb_reduce(ctl_ctx* c, void* comm, ctl_pixel* d_fb, uint64_t n_pixels, int32_t root,
                                 void* stream) {
    if (!c || !comm || (!d_fb && n_pixels)) return CTL_ERR_INVALID;
    if (hipSetDevice(c->device) != hipSuccess) { c->err = "fb_reduce: hipSetDevice failed"; return CTL_ERR_HIP; }
    const size_t count = (size_t)n_pixels * (sizeof(ctl_pixel) / sizeof(float));
    return nccl_status(c, ncclReduce(d_fb, d_fb, count, ncclFloat, ncclSum, root, reinterpret_cast<ncclComm_t>(comm),
                                     reinterpret_cast<hipStream_t>(stream)),
                       "fb_reduce: ncclReduce");
}

CTL_API ctl_status ctl_fb_reduce_all(ctl_ctx* const* ctxs, void* const* comms, ctl_pixel* const* d_fbs, int32_t n,
                                     uint64_t n_pixels, int32_t root, void* const* streams) {
    if (!ctxs || !comms || !d_fbs || n < 1) return CTL_ERR_INVALID;
    const size_t count = (size_t)n_pixels * (sizeof(ctl_pixel) / sizeof(float));
    if (ncclGroupStart() != ncclSuccess) return CTL_ERR_HIP;
    ctl_status st = CTL_OK;
    for (int i = 0; i < n && st == CTL_OK; i++) {
        ctl_ctx* c = ctxs[i];
        if (!c || !comms[i]) { st = CTL_ERR_INVALID; break; }
        if (hipSetDevice(c->device) != hipSuccess) { c->err = "fb_reduce_all: hipSetDevice failed"; st = CTL_ERR_HIP; break; }
        st = nccl_status(c, ncclReduce(d_fbs[i], d_fbs[i], count, ncclFloat, ncclSum, root,
                                       reinterpret_cast<ncclComm_t>(comms[i]),
                                       reinterpret_cast<hipStream_t>(streams ? streams[i] : nullptr)),
                         "fb_reduce_all: ncclReduce");
    }
    const ncclResult_t g = ncclGroupEnd();
    if (st != CTL_OK) return st;
    return nccl_status(ctxs[0], g, "fb_reduce_all: ncclGroupEnd");
}

}  // extern "C"
