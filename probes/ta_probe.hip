// ta_probe.hip — cost model of the vector-memory address path (TA) for the
// traversal's node fetch.  Each lane walks a dependent chain of 128-B nodes
// (random, L2-resident); only lanes < A of every wave are active.
//   D  : direct fetch, 7 x 16-B loads per active lane (the wide-node step);
//   T7 : transposed fetch, the A*7 chunks spread over all 64 lanes
//        (ceil(7A/64) loads), handed back through LDS;
//   T8 : the same with 8 lanes per node (whole 128-B line per 8 lanes).
// Prints ns per wave-step for each (variant, A).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int kNodes = 1 << 14;   // 2 MiB of nodes: L2-resident
constexpr int kBlock = 256;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

template <int V>
__global__ __launch_bounds__(kBlock) void probe(const float4* __restrict__ nodes, int iters, int A, uint32_t* out) {
    extern __shared__ float4 lds[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    float4* buf = lds + wave * 64 * 8;
    uint32_t idx = mix(blockIdx.x * kBlock + threadIdx.x) & (kNodes - 1);
    uint32_t acc = 0;
    const bool act = lane < A;
    for (int it = 0; it < iters; it++) {
        float4 c[7];
        if (V == 0 || V == 5) {
            if (act) {
                // V 5: every lane of the wave reads lane 0's node (one line per instruction)
                const uint32_t ni = V == 5 ? (uint32_t)__shfl((int)idx, 0) : idx;
                const float4* n = nodes + (size_t)ni * 8;
#pragma unroll
                for (int k = 0; k < 7; k++) c[k] = n[k];
            }
        } else if (V == 3 || V == 4) {
            // 3: clamped register staging (every lane loads every round); 4: LDS-DMA
            const int nch = A * 7;
#pragma unroll
            for (int q = 0; q < 7; q++) {
                if (q * 64 < nch) {
                    int j = q * 64 + lane;
                    if (V == 3) j = min(j, nch - 1);
                    const int owner = j / 7;
                    const int k = j - owner * 7;
                    const uint32_t ni = (uint32_t)__shfl((int)idx, owner & 63);
                    if (V == 3) {
                        buf[q * 64 + lane] = nodes[(size_t)ni * 8 + k];
                    } else if (j < nch) {
                        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(nodes + (size_t)ni * 8 + k),
                                                         (__attribute__((address_space(3))) void*)(buf + q * 64), 16, 0, 0);
                    }
                }
            }
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            if (act) {
#pragma unroll
                for (int k = 0; k < 7; k++) c[k] = buf[lane * 7 + k];
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else {
            const int per = V == 1 ? 7 : 8;
            const int nch = A * per;
            for (int base = 0; base < nch; base += 64) {
                const int j = base + lane;
                const int owner = j / per;
                const int k = j - owner * per;
                const uint32_t ni = (uint32_t)__shfl((int)idx, owner & 63);
                if (j < nch) buf[j] = nodes[(size_t)ni * 8 + k];
            }
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            if (act) {
#pragma unroll
                for (int k = 0; k < 7; k++) c[k] = buf[lane * per + k];
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        if (act) {
            uint32_t h = 0;
#pragma unroll
            for (int k = 0; k < 7; k++) h += __float_as_uint(c[k].x) ^ __float_as_uint(c[k].w);
            acc += h;
            idx = mix(h + idx) & (kNodes - 1);
        }
    }
    if (acc == 0x12345678u) out[0] = idx;
}

int main() {
    std::vector<float4> h((size_t)kNodes * 8);
    for (size_t i = 0; i < h.size(); i++) {
        uint32_t r = (uint32_t)(i * 2654435761u);
        h[i] = make_float4(__builtin_bit_cast(float, r), 1.0f, 2.0f, __builtin_bit_cast(float, r ^ 0x5555u));
    }
    float4* d; uint32_t* o;
    CHECK(hipMalloc(&d, h.size() * sizeof(float4)));
    CHECK(hipMalloc(&o, 4));
    CHECK(hipMemcpy(d, h.data(), h.size() * sizeof(float4), hipMemcpyHostToDevice));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int blocks = cus * 4;   // 16 waves per CU
    const int iters = 400;
    const size_t lds = 4 * 64 * 8 * sizeof(float4);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    const int As[] = {64, 32, 26, 16, 8};
    const char* names[] = {"D", "T7", "T8", "T7C", "T7D", "DSAME"};
    for (int v = 0; v < 6; v++) {
        if (v == 2) continue;
        for (int A : As) {
            auto launch = [&]() {
                if (v == 0) probe<0><<<blocks, kBlock, lds>>>(d, iters, A, o);
                else if (v == 1) probe<1><<<blocks, kBlock, lds>>>(d, iters, A, o);
                else if (v == 2) probe<2><<<blocks, kBlock, lds>>>(d, iters, A, o);
                else if (v == 3) probe<3><<<blocks, kBlock, lds>>>(d, iters, A, o);
                else if (v == 4) probe<4><<<blocks, kBlock, lds>>>(d, iters, A, o);
                else probe<5><<<blocks, kBlock, lds>>>(d, iters, A, o);
            };
            launch();
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0));
            for (int r = 0; r < 5; r++) launch();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double steps = 5.0 * blocks * 4 * iters;   // wave-steps
            printf("%-3s A=%2d  %.3f ms  %.3f ns/wave-step (chip)  %.1f cyc/wave-step/CU @2.4GHz\n", names[v], A, ms / 5,
                   ms * 1e6 / steps, ms * 1e-3 / steps * cus * 2.4e9);
        }
    }
    return 0;
}
