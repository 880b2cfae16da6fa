// common.h — device pieces shared by the megakernel (ctl_trace.hip) and the
// wavefront pipeline (wavefront.hip): pass parameters, the SequenceSampler,
// sensor rays, AddSample, and the context structure of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "traverse.h"

namespace ctl {

constexpr int kBlock = 256;

struct PathParams {
    uint32_t width, height;
    int32_t max_path_length, rr_start_depth;
    uint32_t tile_size, tiles_x, num_tiles, num_ranks, rank;
    uint32_t nseq, len;
    int32_t shadow_any_hit;
    bool half_quirk;
};

struct SamplerDev {   // SequenceSampler (Kernel/Sampler_device.h:59-113)
    const float* s1;
    const float2* s2;
    uint32_t nseq, len, a, b;   // a = idx % nseq, b = (idx / nseq) % nseq
    uint32_t d1, d2;
    __device__ __forceinline__ void init(const float* t1, const float2* t2, const PathParams& P, uint32_t idx,
                                         uint32_t c1, uint32_t c2) {
        s1 = t1; s2 = t2; nseq = P.nseq; len = P.len;
        a = idx % P.nseq; b = (idx / P.nseq) % P.nseq;
        d1 = c1; d2 = c2;
    }
    __device__ __forceinline__ float next1() {
        uint32_t k = d1 % len;
        float val = 0.0f;
        val += s1[k * nseq + a];
        val += s1[k * nseq + b];
        d1++;
        return fracf_ref(val);
    }
    __device__ __forceinline__ f2 next2() {
        uint32_t k = d2 % len;
        float2 p = s2[k * nseq + a], q = s2[k * nseq + b];
        float x = 0.0f, y = 0.0f;
        x += p.x; y += p.y;
        x += q.x; y += q.y;
        d2++;
        return mk2(fracf_ref(x), fracf_ref(y));
    }
};

struct LutDecode {
    const float4* lut;
    __device__ __forceinline__ f3 operator()(uint32_t c) const { float4 q = lut[c]; return mk3(q.x, q.y, q.z); }
};

__device__ __forceinline__ m44 load_m44(const float4* M) {
    float4 r0 = M[0], r1 = M[1], r2 = M[2], r3 = M[3];
    m44 m;
    m.d[0] = r0.x; m.d[1] = r0.y; m.d[2] = r0.z; m.d[3] = r0.w;
    m.d[4] = r1.x; m.d[5] = r1.y; m.d[6] = r1.z; m.d[7] = r1.w;
    m.d[8] = r2.x; m.d[9] = r2.y; m.d[10] = r2.z; m.d[11] = r2.w;
    m.d[12] = r3.x; m.d[13] = r3.y; m.d[14] = r3.z; m.d[15] = r3.w;
    return m;
}

__device__ __forceinline__ void wave_add_u64(unsigned long long* dst, uint64_t v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(dst, (unsigned long long)v);
}

// work item g -> pixel of the owned tiles (tile_id % num_ranks == rank); each
// wave covers an 8x8 pixel block so primary rays in a wave are coherent.
__device__ __forceinline__ bool work_pixel(const PathParams& P, uint64_t g, uint32_t& px, uint32_t& py) {
    const uint32_t perTile = P.tile_size * P.tile_size;
    const uint32_t j = (uint32_t)(g / perTile), w = (uint32_t)(g % perTile);
    const uint32_t tile = j * P.num_ranks + P.rank;
    if (tile >= P.num_tiles) return false;
    const uint32_t groupsPerRow = P.tile_size / 8;
    const uint32_t grp = w / 64, lane = w % 64;
    px = (tile % P.tiles_x) * P.tile_size + (grp % groupsPerRow) * 8 + lane % 8;
    py = (tile / P.tiles_x) * P.tile_size + (grp / groupsPerRow) * 8 + lane / 8;
    return px < P.width && py < P.height;
}

// PerspectiveSensor::sampleRayDifferential (SceneTypes/Sensor.cu:130-144), primary ray only
__device__ __forceinline__ void sensor_ray(const DevScene& S, f2 pX, f3& o, f3& d) {
    m44 s2c = to_m44(S.camera.sample_to_camera), tw = to_m44(S.camera.to_world);
    f3 nearP = xform_point(s2c, mk3(pX.x * S.camera.inv_resolution[0], pX.y * S.camera.inv_resolution[1], 0.0f));
    f3 dd = normalize(nearP);
    o = xform_point(tw, mk3s(0.0f));
    d = xform_dir(tw, dd);
}

// Image::AddSample (Engine/Image.cu:22-44); one owner per pixel per pass -> plain RMW
__device__ __forceinline__ void add_sample(ctl_pixel* fb, const PathParams& P, f2 pX, spec col) {
    col.x = tmax(0.0f, col.x); col.y = tmax(0.0f, col.y); col.z = tmax(0.0f, col.z);
    int x = (int)floorf(pX.x), y = (int)floorf(pX.y);
    bool valid = !(isnan(col.x) || isnan(col.y) || isnan(col.z)) && isfinite(col.x) && isfinite(col.y) &&
                 isfinite(col.z) && col.x >= 0.0f && col.y >= 0.0f && col.z >= 0.0f;
    if (x >= 0 && x < (int)P.width && y >= 0 && y < (int)P.height && valid) {
        ctl_pixel* pp = fb + (size_t)y * P.width + x;
        pp->rgb[0] += col.x;
        pp->rgb[1] += col.y;
        pp->rgb[2] += col.z;
        pp->weight_sum += 1.0f;
    }
}

// Wavefront path state, structure of arrays (capacity = paths per pass).
struct WfState {
    float4* o;        // ray origin xyz | w: brdf_pdf
    float4* d;        // ray direction xyz | w: unused
    float4* cl;       // accumulated radiance xyz | w: pX.x
    float4* cf;       // throughput xyz | w: pX.y
    float4* wo;       // persistent BSDF wo xyz | w: last_nor.x
    float2* ln;       // last_nor.yz
    uint4* meta;      // x: pixel idx, y: d1 | d2 << 16, z: depth | specular << 16
    float4* hit;      // t, u, v, tri bits
    uint32_t* hit_node;
    uint32_t* q[2];   // extension-ray queues (path indices), ping-pong
    uint32_t* sq;     // shadow queue (path indices)
    float4* sh_o;     // shadow ray origin | w: tmax (any-hit: dist - eps)
    float4* sh_d;     // shadow ray direction | w: dist
    float4* sh_val;   // contribution to add if unoccluded | w: terminated flag
    uint32_t* sh_occ; // occlusion result
    uint32_t* counts; // [2 * bounce + {0: ext queue, 1: shadow queue}]
    size_t capacity;
};

}  // namespace ctl

struct ctl_ctx {
    int device = 0;
    std::string err;
    std::vector<void*> scene_allocs;
    ctl::DevScene scene{};
    bool has_scene = false;
    bool half_quirk = false;
    uint32_t nseq = 4096, len = 30;
    float* d_s1[2] = {nullptr, nullptr};
    float2* d_s2[2] = {nullptr, nullptr};
    float* h_s1[2] = {nullptr, nullptr};
    float* h_s2[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    int next_buf = 0, active = -1;
    unsigned long long* d_counters = nullptr;   // [0] rays [1] overflow [2..4] stats
    uint32_t* d_powers = nullptr;               // XORWOW step powers for sampler_kernel
    ctl::WfState wf{};
    std::vector<void*> wf_allocs;
    int cu_count = 256;
};

namespace ctl {
// wavefront.hip
int wavefront_pass(ctl_ctx* c, const PathParams& P, ctl_pixel* fb, bool stats, hipStream_t s);
void wavefront_free(ctl_ctx* c);
}
