// image.hip — the final-image stage after accumulation:
//   image_resolve_kernel   copySamplesToOutput + gammaCorrecture   Kernel/ImagePipeline/ImagePipeline.cu:8-21
//                          PixelData::toSpectrum                   Engine/Image.h:21-28
//   variance_add_kernel    PixelVarianceInfo::updateMoments        Kernel/PixelVarianceBuffer.h:22-41
//                          (launched like updateVarianceBuffer,    Kernel/PixelVarianceBuffer.cu:10-37)
//   variance_stats_kernel  computeError / computeVariance / computeAverage, PixelVarianceBuffer.h:43-62
// One thread per pixel, 256-thread blocks; everything is HBM-streaming work
// (28 B in, 4 B out per pixel for the resolve).  fp32, reference op order.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "../../../include/ctl_trace.h"
#include "common.h"

namespace ctl {
namespace {

// toSRGBComponent (Math/Spectrum.cu:229-234)
__device__ __forceinline__ float to_srgb(float v) {
    if (v <= (float)0.0031308) return (float)12.92 * v;
    return (float)1.055 * cr_pow(v, (float)(1.0 / 2.4)) - (float)0.055;
}
// SpectrumConverter::Float3ToCOLORREF (Math/Spectrum.h:521-526)
__device__ __forceinline__ uint32_t to_u8(float x) { return (uint32_t)(unsigned char)(tmin(tmax(x, 0.0f), 1.0f) * 255.0f); }

__global__ __launch_bounds__(kBlock) void image_resolve_kernel(const ctl_pixel* fb, uint32_t n, float splat,
                                                               uint32_t* out) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const ctl_pixel p = fb[i];
    const float weight = p.weight_sum != 0 ? p.weight_sum : 1;
    const spec s = spec_div(mk3(p.rgb[0], p.rgb[1], p.rgb[2]), weight) +
                   mk3(p.rgb_splat[0], p.rgb_splat[1], p.rgb_splat[2]) * splat;
    const float r = to_srgb(s.x), g = to_srgb(s.y), b = to_srgb(s.z);
    out[i] = to_u8(r) | (to_u8(g) << 8) | (to_u8(b) << 16) | (255u << 24);
}

__device__ __forceinline__ float luminance(spec s) { return s.x * 0.212671f + s.y * 0.715160f + s.z * 0.072169f; }

__global__ __launch_bounds__(kBlock) void variance_add_kernel(const ctl_pixel* fb, uint32_t w, uint32_t h, float splat,
                                                              uint32_t tile, uint32_t tiles_x, const uint8_t* flags,
                                                              ctl_pixel_variance* var) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= w * h) return;
    const uint32_t x = i % w, y = i / w;
    const uint8_t f = flags[(y / tile) * tiles_x + x / tile];
    if (!f) return;
    const float samplerPerformed = (float)(char)f;
    const ctl_pixel p = fb[i];
    ctl_pixel_variance v = var[i];
    const spec sum = mk3(p.rgb[0], p.rgb[1], p.rgb[2]) + mk3(p.rgb_splat[0], p.rgb_splat[1], p.rgb_splat[2]) * splat;
    const spec est = spec_div(sum - mk3(v.prev_I[0], v.prev_I[1], v.prev_I[2]), samplerPerformed);
    v.prev_I[0] = sum.x; v.prev_I[1] = sum.y; v.prev_I[2] = sum.z;
    v.weight = p.weight_sum;
    if (v.iterations_done++ % 2 == 1) {
        v.half_buffer[0] += est.x; v.half_buffer[1] += est.y; v.half_buffer[2] += est.z;
    }
    if (samplerPerformed != 0) {   // VarAccumulator += (Math/VarAccumulator.h:26-31)
        const float L = luminance(est);
        v.sum_x += L;
        v.sum_x2 += L * L;
        v.num_samples_var++;
    }
    var[i] = v;
}

__global__ __launch_bounds__(kBlock) void variance_stats_kernel(const ctl_pixel_variance* var, uint64_t n, float* err,
                                                                float* variance, float* average) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const ctl_pixel_variance v = var[i];
    if (err) {
        const spec I = spec_div(mk3(v.prev_I[0], v.prev_I[1], v.prev_I[2]), v.weight);
        const spec A = spec_div(mk3(v.half_buffer[0], v.half_buffer[1], v.half_buffer[2]), float(v.iterations_done / 2));
        const spec d = I - A;
        float s1 = 0.0f; s1 += fabsf(d.x); s1 += fabsf(d.y); s1 += fabsf(d.z);
        float s2 = 0.0f; s2 += I.x; s2 += I.y; s2 += I.z;
        const float e_p = s1 / sqrtf(s2);
        const bool Izero = I.x == 0.0f && I.y == 0.0f && I.z == 0.0f;
        const bool Inan = isnan(I.x) || isnan(I.y) || isnan(I.z), Anan = isnan(A.x) || isnan(A.y) || isnan(A.z);
        err[i] = Izero || Inan || Anan ? 0.0f : tmax(e_p, 1e-2f);
    }
    const float N = (float)v.num_samples_var;
    if (variance) {   // VarianceFromMoments (VarAccumulator.h:7-11)
        const float invN = 1.0f / N;
        variance[i] = (v.sum_x2 - (v.sum_x * v.sum_x) * invN) * invN;
    }
    if (average) average[i] = v.sum_x / N;
}

}  // namespace
}  // namespace ctl

using namespace ctl;

#define CTL_HIP(ctx, call)                                                                 \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess) {                                                            \
            (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);                \
            return CTL_ERR_HIP;                                                            \
        }                                                                                  \
    } while (0)

extern "C" {

CTL_API ctl_status ctl_image_resolve(ctl_ctx* c, const ctl_pixel* fb, uint32_t w, uint32_t h, float splat,
                                     uint32_t* out, void* stream) {
    if (!c || ((!fb || !out) && (uint64_t)w * h)) return CTL_ERR_INVALID;
    const uint64_t n = (uint64_t)w * h;
    if (n == 0) return CTL_OK;
    if (n > 0xffffffffull) { c->err = "image_resolve: image too large"; return CTL_ERR_INVALID; }
    CTL_HIP(c, hipSetDevice(c->device));
    hipLaunchKernelGGL(image_resolve_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), fb, (uint32_t)n, splat, out);
    CTL_HIP(c, hipGetLastError());
    return CTL_OK;
}

CTL_API ctl_status ctl_variance_add_pass(ctl_ctx* c, const ctl_pixel* fb, uint32_t w, uint32_t h, float splat,
                                         uint32_t tile, const uint8_t* tile_samples, ctl_pixel_variance* var,
                                         void* stream) {
    if (!c || !tile || !tile_samples || ((!fb || !var) && (uint64_t)w * h)) return CTL_ERR_INVALID;
    const uint64_t n = (uint64_t)w * h;
    if (n == 0) return CTL_OK;
    if (n > 0xffffffffull) { c->err = "variance_add_pass: image too large"; return CTL_ERR_INVALID; }
    const uint32_t tx = (w + tile - 1) / tile, ty = (h + tile - 1) / tile;
    CTL_HIP(c, hipSetDevice(c->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (c->tile_flags_cap < (size_t)tx * ty) {
        CTL_HIP(c, hipStreamSynchronize(s));
        if (c->d_tile_flags) (void)hipFree(c->d_tile_flags);
        c->d_tile_flags = nullptr;
        c->tile_flags_cap = 0;
        CTL_HIP(c, hipMalloc(&c->d_tile_flags, (size_t)tx * ty));
        c->tile_flags_cap = (size_t)tx * ty;
    }
    // pageable source: the copy completes before the call returns, so the
    // caller may reuse tile_samples immediately
    CTL_HIP(c, hipMemcpyAsync(c->d_tile_flags, tile_samples, (size_t)tx * ty, hipMemcpyHostToDevice, s));
    CTL_HIP(c, hipStreamSynchronize(s));
    hipLaunchKernelGGL(variance_add_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, fb, w, h,
                       splat, tile, tx, c->d_tile_flags, var);
    CTL_HIP(c, hipGetLastError());
    return CTL_OK;
}

CTL_API ctl_status ctl_variance_stats(ctl_ctx* c, const ctl_pixel_variance* var, uint64_t n, float* err,
                                      float* variance, float* average, void* stream) {
    if (!c || (!var && n)) return CTL_ERR_INVALID;
    if (n == 0 || (!err && !variance && !average)) return CTL_OK;
    CTL_HIP(c, hipSetDevice(c->device));
    hipLaunchKernelGGL(variance_stats_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), var, n, err, variance, average);
    CTL_HIP(c, hipGetLastError());
    return CTL_OK;
}

}  // extern "C"
