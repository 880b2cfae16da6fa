// raysort.hip — coherent visit order for the batch traversal (ctl_set_ray_order).
//
// The batch traversal (intersect_kernel: ctl_intersect and the WavefrontPathTracer's
// per-bounce batches, the reference's intersectKernel / DoubleRayBuffer,
// Kernel/TraceHelper.cu:326-746, Kernel/DoubleRayBuffer.h:84-112) fetches rays
// in the caller's order.  Incoherent rays then put ~20 distinct cache lines under
// every wave-level node load (19.6 TA cycles per load).  Here the rays
// of a launch are keyed by (direction octant, Morton code of the origin in the
// scene box) and radix-sorted; the traversal fetches them in key order and
// writes every hit to its own slot, so the results are the caller-order
// results byte for byte (a ray's hit is a function of the ray alone).
//
// Keys: the top `bits` bits of a 31-bit key, shifted down (slots past the
// device-side segment counts get 2^bits and sort last).  Mode 1: octant in bits
// 28-30 of the 31-bit key, a 28-bit origin Morton code below it (9-10 bits per
// axis); mode 2: the Morton code on top, the octant in the 3 low bits.  The sort
// covers bits [0, bits + 1): rocPRIM 7.2's radix sort returns no permutation
// for inputs of at most 2^20 elements when begin_bit > 0
// (probes/rocprim_sort_check.hip, profiles/r05_rocprim_sort_check.txt).
// Order entries name slots: segment 1 slot i -> i, segment 2 slot j -> 2^31 | j.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "common.h"

namespace ctl {

namespace {

__device__ __forceinline__ uint32_t spread3(uint32_t x) {   // 10 bits -> every third bit of 30
    x &= 0x3ffu;
    x = (x | (x << 16)) & 0x030000ffu;
    x = (x | (x << 8)) & 0x0300f00fu;
    x = (x | (x << 4)) & 0x030c30c3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}

__global__ __launch_bounds__(256) void ray_key_kernel(const ctl_ray* rays, uint32_t n, const ctl_ray* rays2, uint32_t n2,
                                                      const uint32_t* dcount, float3 lo, float3 scale, int mode,
                                                      uint32_t bits, uint32_t* keys, uint32_t* vals) {
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k >= n + n2) return;
    const bool second = k >= n;
    const uint32_t j = second ? k - n : k;
    const uint32_t live = dcount ? dcount[second ? 1 : 0] : (second ? n2 : n);
    vals[k] = second ? (0x80000000u | j) : j;
    if (j >= live) {
        keys[k] = 1u << bits;
        return;
    }
    const float4* r4 = reinterpret_cast<const float4*>((second ? rays2 : rays) + j);
    const float4 o = r4[0], d = r4[1];
    const uint32_t oct = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
    auto q = [](float v, float l, float s) {
        const float t = (v - l) * s;   // [0, 1024) inside the box
        return t <= 0.0f ? 0u : (t >= 1023.0f ? 1023u : (uint32_t)t);
    };
    const uint32_t m = spread3(q(o.x, lo.x, scale.x)) | (spread3(q(o.y, lo.y, scale.y)) << 1) |
                       (spread3(q(o.z, lo.z, scale.z)) << 2);   // 30 bits
    const uint32_t m28 = m >> 2;
    const uint32_t key31 = mode == 2 ? ((m28 << 3) | oct) : ((oct << 28) | m28);
    keys[k] = key31 >> (31u - bits);
}

}  // namespace

void raysort_free(ctl_ctx* c) {
    for (void* p : {(void*)c->rs_keys[0], (void*)c->rs_keys[1], (void*)c->rs_vals, (void*)c->rs_order, c->rs_temp})
        if (p) (void)hipFree(p);
    c->rs_keys[0] = c->rs_keys[1] = c->rs_vals = nullptr;
    c->rs_order = nullptr;
    c->rs_temp = nullptr;
    c->rs_cap = 0;
    c->rs_temp_bytes = 0;
}

// Sorted visit order of the n + n2 slots (n, n2: segment sizes or, with dcount,
// their upper bounds); c->rs_order on success.
int sort_rays(ctl_ctx* c, uint32_t n, const ctl_ray* rays, uint32_t n2, const ctl_ray* rays2, const uint32_t* dcount,
              hipStream_t s) {
    const uint32_t total = n + n2;
    if (c->rs_cap < total) {
        raysort_free(c);
        const size_t cap = (size_t)total + total / 4;
        if (hipMalloc(&c->rs_keys[0], cap * 4) != hipSuccess || hipMalloc(&c->rs_keys[1], cap * 4) != hipSuccess ||
            hipMalloc(&c->rs_vals, cap * 4) != hipSuccess || hipMalloc(&c->rs_order, cap * 4) != hipSuccess) {
            raysort_free(c);
            c->err = "ray order: buffer allocation failed";
            return CTL_ERR_NOMEM;
        }
        c->rs_cap = (uint32_t)cap;
    }
    // the sort's temporary storage is laid out for the exact element count and
    // bit range (one queried for another size sorts wrongly: probes/rocprim_sort_check.hip)
    const uint32_t bits = (uint32_t)std::min(31, std::max(1, c->ray_order_bits));
    size_t need = 0;
    if (rocprim::radix_sort_pairs(nullptr, need, c->rs_keys[0], c->rs_keys[1], c->rs_vals, c->rs_order, total, 0u,
                                  bits + 1u, s) != hipSuccess) {
        c->err = "ray order: sort storage query failed";
        return CTL_ERR_HIP;
    }
    if (need > c->rs_temp_bytes) {
        if (c->rs_temp && (hipStreamSynchronize(s) != hipSuccess || hipFree(c->rs_temp) != hipSuccess)) {
            c->err = "ray order: sort storage release failed";
            return CTL_ERR_HIP;
        }
        c->rs_temp = nullptr;
        c->rs_temp_bytes = 0;
        if (hipMalloc(&c->rs_temp, need) != hipSuccess) {
            c->err = "ray order: sort storage allocation failed";
            return CTL_ERR_NOMEM;
        }
        c->rs_temp_bytes = need;
    }
    const float* b = c->scene_box;
    auto inv = [](float l, float h) { return h > l ? 1024.0f / (h - l) : 0.0f; };
    const float3 lo = make_float3(b[0], b[1], b[2]);
    const float3 sc = make_float3(inv(b[0], b[3]), inv(b[1], b[4]), inv(b[2], b[5]));
    hipLaunchKernelGGL(ray_key_kernel, dim3((total + 255) / 256), dim3(256), 0, s, rays, n, rays2, n2, dcount, lo, sc,
                       c->ray_order, bits, c->rs_keys[0], c->rs_vals);
    if (hipGetLastError() != hipSuccess) { c->err = "ray order: key launch failed"; return CTL_ERR_HIP; }
    // the key bits and the empty-slot bit above them
    if (rocprim::radix_sort_pairs(c->rs_temp, need, c->rs_keys[0], c->rs_keys[1], c->rs_vals, c->rs_order, total,
                                  0u, bits + 1u, s) != hipSuccess) {
        c->err = "ray order: radix sort failed";
        return CTL_ERR_HIP;
    }
    return CTL_OK;
}

}  // namespace ctl

using namespace ctl;

extern "C" {

CTL_API ctl_status ctl_set_ray_order(ctl_ctx* c, int32_t mode, int32_t key_bits) {
    if (!c || mode < 0 || mode > 2 || key_bits < 1 || key_bits > 31) return CTL_ERR_INVALID;
    c->ray_order = mode;
    c->ray_order_bits = key_bits;
    return CTL_OK;
}

}  // extern "C"
