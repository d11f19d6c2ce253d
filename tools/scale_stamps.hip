// Phase stamps of the MFMA Lanczos scaler (k_scale_mfma), one line per phase: where a 4K -> 1080p
// dispatch spends its time.  Builds csrc/kernels/pixel.hip with MX_SCALE_STAMPS into a standalone
// program (no Python, no extension):
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form -DMX_SCALE_STAMPS -Icsrc \
//         tools/scale_stamps.hip -o tools/scale_stamps.bin
//   tools/scale_stamps.bin [reps=20] [in_w in_h out_w out_h]
// (the -mllvm flag is the one mxdesk/_build.py compiles pixel.hip with).  Without
// -DMX_SCALE_STAMPS it times the production kernel only (for rocprofv3 --kernel-trace --stats).
//
// Stamps per workgroup (pixel.hip MF_STAMP): realtime at entry / exit (100 MHz, comparable across
// XCDs) and s_memtime between the phases: weights + block 0/1 DMA landed, block 0 products,
// block 1 landed, remaining blocks, epilogue.
#include "../csrc/kernels/pixel.hip"

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

using namespace mx::pix;

static double lanczos3(double x) {
    if (x == 0.0) return 1.0;
    if (x <= -3.0 || x >= 3.0) return 0.0;
    const double px = M_PI * x;
    return 3.0 * std::sin(px) * std::sin(px / 3.0) / (px * px);
}

// the session's table (csrc/runtime/session.cpp make_lanczos_table)
static void table(int in_size, int out_size, std::vector<int>& start, std::vector<float>& weights, int& taps) {
    const double s = (double)in_size / out_size, f = std::max(1.0, s), support = 3.0 * f;
    taps = (int)std::ceil(2.0 * support) + 1;
    start.resize(out_size);
    weights.assign((size_t)out_size * taps, 0.f);
    for (int o = 0; o < out_size; ++o) {
        const double center = (o + 0.5) * s - 0.5;
        const int x0 = (int)std::floor(center - support) + 1;
        start[o] = x0;
        double sum = 0;
        std::vector<double> w(taps);
        for (int k = 0; k < taps; ++k) sum += (w[k] = lanczos3((x0 + k - center) / f));
        for (int k = 0; k < taps; ++k) weights[(size_t)o * taps + k] = (float)(w[k] / sum);
    }
}

static void pct(const char* name, std::vector<double> v, const char* unit) {
    std::sort(v.begin(), v.end());
    auto at = [&](double q) { return v[std::min(v.size() - 1, (size_t)(q * v.size()))]; };
    printf("%-28s min %8.2f  p10 %8.2f  p50 %8.2f  p90 %8.2f  max %8.2f %s\n", name, v.front(), at(0.1), at(0.5),
           at(0.9), v.back(), unit);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const int in_w = argc > 5 ? atoi(argv[2]) : 3840, in_h = argc > 5 ? atoi(argv[3]) : 2160;
    const int out_w = argc > 5 ? atoi(argv[4]) : 1920, out_h = argc > 5 ? atoi(argv[5]) : 1080;
    const int cw = (out_w + 15) / 16 * 16, ch = (out_h + 15) / 16 * 16;
    std::vector<int> x0, y0;
    std::vector<float> wx, wy;
    int tx, ty;
    table(in_w, out_w, x0, wx, tx);
    table(in_h, out_h, y0, wy, ty);
    ScaleFragsHost fr;
    if (!build_scale_frags(in_w, in_h, out_w, out_h, cw, ch, x0, wx, tx, y0, wy, ty, fr)) {
        fprintf(stderr, "geometry outside the MFMA kernel\n");
        return 2;
    }
    LanczosTables t{out_w, out_h, tx, ty, nullptr, nullptr, nullptr, nullptr};
    void* frags = nullptr;
    upload_scale_frags(fr, &frags, t.mf);
    std::vector<uint8_t> host((size_t)in_w * in_h * 4);
    std::mt19937 rng(7);
    for (size_t i = 0; i < host.size(); i += 4) {  // smooth-ish content with noise
        const uint32_t r = rng();
        host[i] = (uint8_t)(r), host[i + 1] = (uint8_t)(r >> 8), host[i + 2] = (uint8_t)(r >> 16), host[i + 3] = 255;
    }
    uint8_t *in = nullptr, *y = nullptr, *uv = nullptr;
    HIP_CHECK(hipMalloc(&in, host.size()));
    HIP_CHECK(hipMalloc(&y, (size_t)cw * ch));
    HIP_CHECK(hipMalloc(&uv, (size_t)cw * ch / 2));
    HIP_CHECK(hipMemcpy(in, host.data(), host.size(), hipMemcpyHostToDevice));
    hipStream_t st;
    HIP_CHECK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) launch_scale_to_nv12(in, in_w * 4, in_w, in_h, t, y, uv, cw, cw, ch, st);
    HIP_CHECK(hipEventRecord(e0, st));
    for (int i = 0; i < reps; ++i) launch_scale_to_nv12(in, in_w * 4, in_w, in_h, t, y, uv, cw, cw, ch, st);
    HIP_CHECK(hipEventRecord(e1, st));
    HIP_CHECK(hipStreamSynchronize(st));
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    const int gx = (cw + 63) / 64, gy = (ch + 31) / 32, nwg = gx * gy;
#ifndef MX_SCALE_STAMPS  // the production kernel: launch timing only (run it under rocprofv3)
    printf("%dx%d -> %dx%d: %d workgroups, lds_cols %d, %.2f us per launch (events, %d back-to-back)\n", in_w, in_h,
           out_w, out_h, nwg, fr.lds_cols, 1e3 * ms / reps, reps);
    HIP_CHECK(hipFree(frags));
    return 0;
#else
    if (nwg > 4096) return 3;
    std::vector<uint64_t> s((size_t)nwg * 8);
    HIP_CHECK(hipMemcpyFromSymbol(s.data(), HIP_SYMBOL(g_scale_stamps), s.size() * 8));
    printf("%dx%d -> %dx%d: %d workgroups, lds_cols %d, %.2f us per launch (events, %d back-to-back)\n", in_w, in_h,
           out_w, out_h, nwg, fr.lds_cols, 1e3 * ms / reps, reps);
    uint64_t r0 = ~0ull, r1 = 0;
    for (int w = 0; w < nwg; ++w) r0 = std::min(r0, s[w * 8 + 0]), r1 = std::max(r1, s[w * 8 + 7]);
    printf("last launch: first entry -> last exit %.2f us (100 MHz realtime)\n", (r1 - r0) / 100.0);
    std::vector<double> ent, ex, life, ph[5];
    for (int w = 0; w < nwg; ++w) {
        const uint64_t* p = &s[w * 8];
        ent.push_back((p[0] - r0) / 100.0);
        ex.push_back((p[7] - r0) / 100.0);
        life.push_back((p[7] - p[0]) / 100.0);
        for (int k = 0; k < 5; ++k) ph[k].push_back((double)(p[k + 2] - p[k + 1]));
    }
    pct("entry (us after first)", ent, "us");
    pct("exit (us after first)", ex, "us");
    pct("lifetime", life, "us");
    const char* names[5] = {"blocks 0/1 landed", "block 0 products", "block 1 landed", "blocks 1.. products", "epilogue"};
    for (int k = 0; k < 5; ++k) pct(names[k], ph[k], "cyc");
    // entry histogram: how many workgroups started in each microsecond
    const int nb = (int)(r1 - r0) / 100 + 1;
    std::vector<int> hist(nb, 0), live(nb, 0);
    for (int w = 0; w < nwg; ++w) {
        hist[std::min(nb - 1, (int)ent[w])]++;
        for (int b = (int)ent[w]; b <= std::min(nb - 1, (int)ex[w]); ++b) live[b]++;
    }
    printf("us : started / resident\n");
    for (int b = 0; b < nb; ++b) printf("%3d : %4d / %4d\n", b, hist[b], live[b]);
    HIP_CHECK(hipFree(frags));
    return 0;
#endif
}
