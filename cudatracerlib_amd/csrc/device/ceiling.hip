// ceiling.hip — measured ceilings for the roofline of the traversal kernels
// ("record the measured STREAM-like read BW on the box as the
// practical ceiling"), built as libctl_ceiling.so beside the product library.
// Measurement only: nothing in libctl_trace.so calls it.
//
//   hbm_read    STREAM-like read of a buffer far larger than L2 + MALL: every lane
//               streams 16-B loads, four in flight per iteration, a grid-stride
//               loop over the whole buffer; GB/s of the fastest repetition.
//   node_chain  the traversal's dependent fetch chain without its arithmetic:
//               each active lane walks random 128-B nodes, one step = the wide
//               node's seven 16-B loads (traverse.h), the next node a hash of the
//               loaded bytes, so step k+1 cannot issue before step k lands.  A
//               active lanes of every wave (the path kernel's measured lane
//               activity), W waves per SIMD, each lane on its own chain or all
//               lanes of a wave on one (coherent rays share the top of the tree),
//               the node array L1-resident (16 KiB), L2-resident (2 MiB: the path
//               kernel's 99 % L2 hit rate) or the C3 wide tree's size (0.54 GB:
//               every step a far fetch).  Result: lane node steps per second.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(kBlock) void fill_kernel(uint4* p, uint64_t n, uint32_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        const uint32_t a = mix32((uint32_t)i ^ seed), b = mix32(a + 0x9e3779b9u);
        p[i] = make_uint4(a, b, mix32(b), mix32(a ^ 0x5bd1e995u));
    }
}

__global__ __launch_bounds__(kBlock) void hbm_read_kernel(const uint4* __restrict__ p, uint64_t n, uint32_t* out) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    uint64_t i = blockIdx.x * (uint64_t)kBlock + threadIdx.x;
    uint32_t acc = 0;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
        acc ^= a.x ^ a.w ^ b.y ^ b.z ^ c.x ^ c.w ^ d.y ^ d.z;
    }
    for (; i < n; i += stride) acc ^= p[i].x;
    if (acc == 0x9e3779b9u) out[0] = acc;   // never true in practice; keeps the loads
}

__global__ __launch_bounds__(kBlock) void node_chain_kernel(const uint4* __restrict__ nodes, uint32_t mask,
                                                            int steps, int active, int share, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    if (lane >= active) return;
    // lanes in groups of `share` walk the same chain (share 64: the wave's active
    // lanes read one node per step, as coherent rays near the root do)
    uint32_t idx = mix32(blockIdx.x * kBlock + (threadIdx.x & ~63) + lane / share) & mask;
    uint32_t acc = 0;
    for (int s = 0; s < steps; s++) {
        const uint4* q = nodes + (size_t)idx * 8;
        uint4 c[7];
#pragma unroll
        for (int k = 0; k < 7; k++) c[k] = q[k];
        uint32_t h = 0;
#pragma unroll
        for (int k = 0; k < 7; k++) h += c[k].x ^ c[k].w;
        acc += h;
        idx = mix32(h + idx) & mask;
    }
    if (acc == 0x12345678u) out[0] = idx;
}

struct Dev {
    int prev = -1;
    explicit Dev(int d) { hipGetDevice(&prev); hipSetDevice(d); }
    ~Dev() { if (prev >= 0) hipSetDevice(prev); }
};

// best and mean of `reps` timed launches (after one warm-up); -1 on a HIP error
template <class F>
int time_reps(int reps, F launch, float* best_ms, float* mean_ms) {
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -1;
    launch();
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    float best = 1e30f, sum = 0.0f;
    for (int r = 0; r < reps; r++) {
        hipEventRecord(e0);
        launch();
        hipEventRecord(e1);
        if (hipEventSynchronize(e1) != hipSuccess) return -1;
        float ms = 0.0f;
        hipEventElapsedTime(&ms, e0, e1);
        best = std::min(best, ms);
        sum += ms;
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    *best_ms = best;
    *mean_ms = sum / reps;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace

extern "C" {

// STREAM-like HBM read of `bytes` (rounded down to 16 B): out[0] = best GB/s,
// out[1] = mean GB/s over `reps`.  Returns 0, or -1 on a HIP error.
__attribute__((visibility("default"))) int ctl_ceiling_hbm_read(int device, uint64_t bytes, int reps, double* out) {
    if (!out || bytes < (1u << 20) || reps < 1) return -1;
    Dev g(device);
    const uint64_t n = bytes / 16;
    uint4* p = nullptr;
    uint32_t* o = nullptr;
    if (hipMalloc(&p, n * 16) != hipSuccess) return -1;
    if (hipMalloc(&o, 4) != hipSuccess) { hipFree(p); return -1; }
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    const int blocks = std::max(1, cus) * 8;   // 8 blocks of 4 waves per CU
    hipLaunchKernelGGL(fill_kernel, dim3(blocks), dim3(kBlock), 0, 0, p, n, 0x5EEDu);
    float best = 0, mean = 0;
    const int r = time_reps(reps, [&] { hipLaunchKernelGGL(hbm_read_kernel, dim3(blocks), dim3(kBlock), 0, 0, p, n, o); },
                            &best, &mean);
    hipFree(p);
    hipFree(o);
    if (r) return -1;
    out[0] = (double)(n * 16) / (best * 1e-3) / 1e9;
    out[1] = (double)(n * 16) / (mean * 1e-3) / 1e9;
    return 0;
}

// Dependent walks over `bytes` (rounded down to a power of two) of random 128-B
// nodes (seven 16-B loads per step), `active` lanes of 64 per wave, lanes in
// groups of `share` on one chain, `waves_per_simd` waves on each SIMD (4 SIMDs
// per CU), `steps` steps per lane.  out[0] = lane node steps per second (best
// of `reps`), out[1] = ns per wave step on one SIMD (best), out[2] = the node
// array's bytes.  Returns 0 or -1.
__attribute__((visibility("default"))) int ctl_ceiling_node_chain(int device, uint64_t bytes, int active, int share,
                                                                  int waves_per_simd, int steps, int reps,
                                                                  double* out) {
    if (!out || bytes < 128 * 2 || active < 1 || active > 64 || share < 1 || share > 64 || waves_per_simd < 1 ||
        waves_per_simd > 8 || steps < 1 || reps < 1)
        return -1;
    Dev g(device);
    uint64_t n_nodes64 = 1;
    while (n_nodes64 * 2 <= bytes / 128) n_nodes64 *= 2;
    if (n_nodes64 > 0x80000000ull) return -1;
    const uint32_t n_nodes = (uint32_t)n_nodes64;
    uint4* p = nullptr;
    uint32_t* o = nullptr;
    if (hipMalloc(&p, (size_t)n_nodes * 128) != hipSuccess) return -1;
    if (hipMalloc(&o, 4) != hipSuccess) { hipFree(p); return -1; }
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    cus = std::max(1, cus);
    hipLaunchKernelGGL(fill_kernel, dim3(cus * 8), dim3(kBlock), 0, 0, p, (uint64_t)n_nodes * 8, 0xC0FFEEu);
    // one 256-thread block = 4 waves = one wave per SIMD of a CU
    const int blocks = cus * waves_per_simd;
    float best = 0, mean = 0;
    const int r = time_reps(reps, [&] {
        hipLaunchKernelGGL(node_chain_kernel, dim3(blocks), dim3(kBlock), 0, 0, p, n_nodes - 1, steps, active, share,
                           o);
    }, &best, &mean);
    hipFree(p);
    hipFree(o);
    if (r) return -1;
    const double lane_steps = (double)blocks * 4.0 * active * steps;
    out[0] = lane_steps / (best * 1e-3);
    out[1] = best * 1e6 / ((double)steps * waves_per_simd);   // ns per wave step on one SIMD
    out[2] = (double)n_nodes * 128.0;
    return 0;
}

}  // extern "C"
