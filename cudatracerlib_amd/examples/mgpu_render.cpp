// mgpu_render.cpp — one process drives every visible GPU through the C ABI
// alone (no torch): the C++ caller's multi-GPU path of SURVEY.md §8e.
//
//   per GPU i (rank i of N):  ctl_create(i), ctl_scene_upload of one host
//   compile, a framebuffer; every step renders N progressive passes of the
//   rank's tiles (ctl_render_passes, num_ranks = N, rank = i; weak scaling:
//   per-GPU work is fixed); after the last step one grouped RCCL reduce
//   (ctl_fb_reduce_all) sums the rank framebuffers into an image buffer on
//   GPU 0.  The result is the 1-GPU framebuffer of the same passes bit for bit.
//   --reduce-every 1 reduces after every step instead (a progressive preview;
//   the rank framebuffers are only read, so the last reduce is the same image).
//
// usage: mgpu_render [--config C] [--scale S] [--width W] [--height H]
//                    [--steps K] [--devices N] [--reduce-every R] [--out file]
// Prints one line: devices, passes, rays, seconds, Mrays/s.  --out writes
// GPU 0's reduced PixelData framebuffer (W*H*7 floats).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ctl_trace.h"

#define CHECK_CTL(ctx, call)                                                                  \
    do {                                                                                      \
        ctl_status st_ = (call);                                                              \
        if (st_ != CTL_OK) {                                                                  \
            std::fprintf(stderr, "%s failed (%d): %s\n", #call, (int)st_, ctl_last_error(ctx)); \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)
#define CHECK_HIP(call)                                                                       \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s failed: %s\n", #call, hipGetErrorString(e_));            \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

int main(int argc, char** argv) {
    int config = 2, steps = 2, ndev = 0, reduce_every = 0;
    double scale = 0.25;
    uint32_t width = 320, height = 180;
    std::string out;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string a = argv[i];
        if (a == "--config") config = std::atoi(argv[i + 1]);
        else if (a == "--scale") scale = std::atof(argv[i + 1]);
        else if (a == "--width") width = (uint32_t)std::atoi(argv[i + 1]);
        else if (a == "--height") height = (uint32_t)std::atoi(argv[i + 1]);
        else if (a == "--steps") steps = std::atoi(argv[i + 1]);
        else if (a == "--devices") ndev = std::atoi(argv[i + 1]);
        else if (a == "--reduce-every") reduce_every = std::atoi(argv[i + 1]);
        else if (a == "--out") out = argv[i + 1];
        else { std::fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
    }
    int visible = 0;
    CHECK_HIP(hipGetDeviceCount(&visible));
    if (ndev <= 0 || ndev > visible) ndev = visible;
    if (ndev < 1) { std::fprintf(stderr, "no GPU\n"); return 1; }

    // one host compile, uploaded to every GPU (the scene is replicated)
    ctl_host_scene* hs = ctl_host_scene_create();
    ctl_scene_desc desc;
    if (!hs || ctl_host_scene_generate(hs, config, scale, width, height) != CTL_OK ||
        ctl_host_scene_compile(hs, 0, &desc) != CTL_OK) {
        std::fprintf(stderr, "scene: %s\n", ctl_host_last_error());
        return 1;
    }
    std::vector<ctl_ctx*> ctx((size_t)ndev, nullptr);
    std::vector<ctl_pixel*> fb((size_t)ndev, nullptr);
    std::vector<hipStream_t> stream((size_t)ndev, nullptr);
    const size_t npx = (size_t)width * height;
    for (int i = 0; i < ndev; i++) {
        ctx[(size_t)i] = ctl_create(i);
        if (!ctx[(size_t)i]) { std::fprintf(stderr, "ctl_create(%d): %s\n", i, ctl_last_error(nullptr)); return 1; }
        CHECK_CTL(ctx[(size_t)i], ctl_scene_upload(ctx[(size_t)i], &desc));
        CHECK_HIP(hipSetDevice(i));
        CHECK_HIP(hipStreamCreateWithFlags(&stream[(size_t)i], hipStreamNonBlocking));
        CHECK_HIP(hipMalloc(&fb[(size_t)i], npx * sizeof(ctl_pixel)));
        CHECK_HIP(hipMemsetAsync(fb[(size_t)i], 0, npx * sizeof(ctl_pixel), stream[(size_t)i]));
        CHECK_CTL(ctx[(size_t)i], ctl_reset_rays(ctx[(size_t)i], stream[(size_t)i]));
    }
    ctl_pixel* image = nullptr;   // the reduced image, on GPU 0
    CHECK_HIP(hipSetDevice(0));
    CHECK_HIP(hipMalloc(&image, npx * sizeof(ctl_pixel)));
    std::vector<void*> comm((size_t)ndev, nullptr);
    if (ctl_comm_init_all(comm.data(), ndev, nullptr) != CTL_OK) { std::fprintf(stderr, "ctl_comm_init_all failed\n"); return 1; }
    for (int i = 0; i < ndev; i++) CHECK_CTL(ctx[(size_t)i], ctl_sync(ctx[(size_t)i], stream[(size_t)i]));

    std::vector<void*> sv(stream.begin(), stream.end());
    std::vector<const ctl_pixel*> cfb(fb.begin(), fb.end());
    const auto t0 = std::chrono::steady_clock::now();
    for (int s = 0; s < steps; s++) {
        for (int i = 0; i < ndev; i++) {   // asynchronous: all GPUs render at once
            ctl_pt_params p;
            std::memset(&p, 0, sizeof(p));
            p.direct = 1; p.max_path_length = 50; p.rr_start_depth = 5; p.shadow_any_hit = 1;
            p.tile_size = 64; p.num_ranks = (uint32_t)ndev; p.rank = (uint32_t)i; p.flags = 0;
            CHECK_CTL(ctx[(size_t)i], ctl_render_passes(ctx[(size_t)i], &p, (uint64_t)s * ndev, (uint32_t)ndev,
                                                        fb[(size_t)i], stream[(size_t)i]));
        }
        if ((reduce_every > 0 && (s + 1) % reduce_every == 0) || s + 1 == steps) {
            if (ctl_fb_reduce_all(ctx.data(), comm.data(), cfb.data(), image, ndev, npx, 0, sv.data()) != CTL_OK) {
                std::fprintf(stderr, "ctl_fb_reduce_all: %s\n", ctl_last_error(ctx[0]));
                return 1;
            }
        }
    }
    uint64_t rays = 0;
    for (int i = 0; i < ndev; i++) {
        CHECK_CTL(ctx[(size_t)i], ctl_sync(ctx[(size_t)i], stream[(size_t)i]));   // also reports stack overflows
        rays += ctl_rays_traced(ctx[(size_t)i]);
    }
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("devices %d passes %d rays %llu seconds %.6f mrays_s %.3f\n", ndev, steps * ndev,
                (unsigned long long)rays, sec, (double)rays / sec * 1e-6);
    if (!out.empty()) {
        std::vector<ctl_pixel> h(npx);
        CHECK_HIP(hipSetDevice(0));
        CHECK_HIP(hipMemcpy(h.data(), image, npx * sizeof(ctl_pixel), hipMemcpyDeviceToHost));
        FILE* f = std::fopen(out.c_str(), "wb");
        if (!f || std::fwrite(h.data(), sizeof(ctl_pixel), npx, f) != npx) { std::fprintf(stderr, "write %s failed\n", out.c_str()); return 1; }
        std::fclose(f);
    }
    for (int i = 0; i < ndev; i++) {
        ctl_comm_destroy(comm[(size_t)i]);
        (void)hipSetDevice(i);
        (void)hipFree(fb[(size_t)i]);
        (void)hipStreamDestroy(stream[(size_t)i]);
        ctl_destroy(ctx[(size_t)i]);
    }
    (void)hipSetDevice(0);
    (void)hipFree(image);
    ctl_host_scene_destroy(hs);
    return 0;
}
