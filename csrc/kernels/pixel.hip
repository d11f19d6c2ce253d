// Pixel kernels on gfx950: synthetic desktop renderer (C40), BT.709 BGRx->NV12 colour
// conversion (C42, replaces the NVRTC-compiled `cudaconvert` of the reference's GStreamer
// nvcodec pipeline -- Dockerfile:469-470), fused LDS-tiled Lanczos-3 scale + CSC, and the
// tiled-wall composite (K7).
//
// Memory shapes: every thread of the CSC kernel owns a 4x2 pixel block -> two 16-byte
// BGRx loads, two 4-byte Y stores and one 4-byte interleaved-UV store (Guideline 13).
// The scaler stages its input footprint in LDS once and runs both filter passes out of
// LDS (each input pixel is reused by ~6 horizontal and ~6 vertical taps).
#include <hip/hip_runtime.h>
#include <math.h>

#include <stdexcept>

#include "pixel.h"

namespace mx {
namespace pix {

namespace {

__device__ __forceinline__ uint32_t hash3(uint32_t x, uint32_t y, uint32_t z) {
    uint32_t h = x * 0x8da6b343u ^ y * 0xd8163841u ^ z * 0xcb1ab31fu;
    h ^= h >> 15;
    h *= 0x2c1b3c6du;
    h ^= h >> 12;
    h *= 0x297a2d39u;
    h ^= h >> 15;
    return h;
}

__device__ __forceinline__ uint32_t bgrx(int r, int g, int b) {
    r = r < 0 ? 0 : (r > 255 ? 255 : r);
    g = g < 0 ? 0 : (g > 255 ? 255 : g);
    b = b < 0 ? 0 : (b > 255 ? 255 : b);
    return (uint32_t)b | ((uint32_t)g << 8) | ((uint32_t)r << 16) | 0xff000000u;
}

// glxgears-like gear: inside test + shade.  (gx, gy) relative to gear centre.
__device__ __forceinline__ bool gear_hit(float gx, float gy, float inner, float outer, float depth, int teeth,
                                         float angle, float* shade) {
    const float r = sqrtf(gx * gx + gy * gy);
    const float r2 = outer + depth * 0.5f;
    if (r > r2 || r < inner) return false;
    const float r1 = outer - depth * 0.5f;
    float th = atan2f(gy, gx) - angle;
    const float period = 6.28318531f / teeth;
    float ph = th / period;
    ph -= floorf(ph);
    // trapezoid tooth: rises over [0,.25], flat [.25,.5], falls [.5,.75]
    float tooth;
    if (ph < 0.25f)
        tooth = ph * 4.f;
    else if (ph < 0.5f)
        tooth = 1.f;
    else if (ph < 0.75f)
        tooth = (0.75f - ph) * 4.f;
    else
        tooth = 0.f;
    const float rmax = r1 + (r2 - r1) * tooth;
    if (r > rmax) return false;
    // fake lighting: brighter towards the upper-left, darker bands near edges
    const float edge = fminf(r - inner, rmax - r);
    const float light = 0.55f + 0.45f * (-(gx + gy) / (1.4142f * (r + 1e-3f)));
    *shade = fminf(1.f, light * (edge < 0.12f ? 0.7f : 1.f));
    return true;
}

__device__ __attribute__((noinline)) uint32_t static_px(int gx, int gy, const SynthParams& p);

// Axis-aligned bounds of everything animated (barcode, cursor, moving window, gears,
// terminal, noise panel); outside them desktop_px() == static_px().
struct DynBoxes {
    int x0[6], y0[6], x1[6], y1[6];
};
__device__ __forceinline__ DynBoxes dyn_boxes(const SynthParams& p) {
    const int W = p.wall_w, H = p.wall_h;
    DynBoxes b;
    b.x0[0] = kBarX - kBarCell; b.y0[0] = kBarY - kBarCell;
    b.x1[0] = kBarX + 33 * kBarCell; b.y1[0] = kBarY + 3 * kBarCell;
    b.x0[1] = p.cursor_x >= 0 ? p.cursor_x : 0; b.y0[1] = p.cursor_y;
    b.x1[1] = p.cursor_x >= 0 ? p.cursor_x + 12 : 0; b.y1[1] = p.cursor_y + 19;
    const int mw = W / 8 > 48 ? W / 8 : 48, mh = H / 8 > 32 ? H / 8 : 32;
    b.x0[2] = (int)(W * 0.5f + W * 0.18f * sinf(p.t * 0.7f)) - mw / 2;
    b.y0[2] = (int)(H * 0.62f + H * 0.12f * sinf(p.t * 1.1f)) - mh / 2;
    b.x1[2] = b.x0[2] + mw; b.y1[2] = b.y0[2] + mh;
    b.x0[3] = (int)(W * 0.55f); b.y0[3] = (int)(H * 0.10f);
    b.x1[3] = b.x0[3] + (int)(W * 0.38f); b.y1[3] = b.y0[3] + (int)(H * 0.50f);
    b.x0[4] = (int)(W * 0.04f); b.y0[4] = (int)(H * 0.10f);
    b.x1[4] = b.x0[4] + (int)(W * 0.42f); b.y1[4] = b.y0[4] + (int)(H * 0.38f);
    b.x0[5] = (int)(W * 0.04f); b.y0[5] = (int)(H * 0.55f);
    b.x1[5] = p.noise ? b.x0[5] + (int)(W * 0.16f) : b.x0[5]; b.y1[5] = b.y0[5] + (int)(H * 0.22f);
    return b;
}
// Whether any of pixels [gx, gx+n) of row gy lies in an animated element's bounds.
// (2-pixel margin: the moving window's float position may round differently here than in
// desktop_px() under FMA contraction; margin pixels are rendered exactly, not copied)
__device__ __forceinline__ bool in_dyn(const DynBoxes& b, int gx, int n, int gy) {
    bool hit = false;
#pragma unroll
    for (int k = 0; k < 6; ++k)
        hit |= b.x1[k] > b.x0[k] && gy >= b.y0[k] - 2 && gy < b.y1[k] + 2 && gx + n > b.x0[k] - 2 && gx < b.x1[k] + 2;
    return hit;
}

__device__ uint32_t desktop_px(int gx, int gy, const SynthParams& p) {
    const int W = p.wall_w, H = p.wall_h;
    // ---- barcode (frame id + timestamp), always on top
    if (gy >= kBarY - kBarCell && gy < kBarY + 2 * kBarCell + kBarCell && gx >= kBarX - kBarCell &&
        gx < kBarX + 32 * kBarCell + kBarCell) {
        const int cx = (gx - kBarX), cy = (gy - kBarY);
        if (cx < 0 || cy < 0 || cx >= 32 * kBarCell || cy >= 2 * kBarCell) return bgrx(96, 96, 96);  // quiet zone
        const int bit = 31 - cx / kBarCell;
        const uint32_t word = (cy / kBarCell) == 0 ? p.frame_id : p.timestamp_us;
        const int v = ((word >> bit) & 1) ? 255 : 0;
        return bgrx(v, v, v);
    }
    // ---- cursor (arrow, 12x19)
    if (p.cursor_x >= 0) {
        const int dx = gx - p.cursor_x, dy = gy - p.cursor_y;
        if (dx >= 0 && dy >= 0 && dy < 19 && dx <= dy * 2 / 3 && dx < 12) {
            const bool border = dx == 0 || dx == dy * 2 / 3 || dy == 18;
            return border ? bgrx(0, 0, 0) : bgrx(255, 255, 255);
        }
    }
    // ---- moving window (Lissajous path, sub-pixel speeds)
    {
        const int mw = W / 8 > 48 ? W / 8 : 48, mh = H / 8 > 32 ? H / 8 : 32;
        const float cxm = W * 0.5f, cym = H * 0.62f;
        const int wx = (int)(cxm + W * 0.18f * sinf(p.t * 0.7f)) - mw / 2;
        const int wy = (int)(cym + H * 0.12f * sinf(p.t * 1.1f)) - mh / 2;
        if (gx >= wx && gx < wx + mw && gy >= wy && gy < wy + mh) {
            if (gy - wy < 10) return bgrx(40, 90, 200);
            const int u = (gx - wx) * 255 / mw, v = (gy - wy) * 255 / mh;
            return bgrx(230 - v / 4, 200 + u / 8, 120 + u / 3);
        }
    }
    // ---- gears window
    {
        const int x0 = (int)(W * 0.55f), y0 = (int)(H * 0.10f);
        const int ww = (int)(W * 0.38f), wh = (int)(H * 0.50f);
        if (gx >= x0 && gx < x0 + ww && gy >= y0 && gy < y0 + wh) {
            if (gy - y0 < 12) return bgrx(60, 60, 70);  // title bar
            const float s = 16.f / (ww < wh ? ww : wh);
            const float sx = (gx - x0 - ww * 0.5f) * s, sy = -((gy - y0 - 6) - (wh - 12) * 0.5f) * s - 1.0f;
            const float a = p.t * 1.5707963f;  // 90 deg/s like glxgears' default speed order
            float sh;
            if (gear_hit(sx + 3.0f, sy + 2.0f, 1.0f, 4.0f, 0.7f, 20, a, &sh))
                return bgrx((int)(204 * sh), (int)(25 * sh), 0);
            if (gear_hit(sx - 3.1f, sy + 2.0f, 0.5f, 2.0f, 0.7f, 10, -2.f * a - 0.157f, &sh))
                return bgrx(0, (int)(204 * sh), (int)(50 * sh));
            if (gear_hit(sx + 3.1f, sy - 4.2f, 1.3f, 2.0f, 0.7f, 10, -2.f * a - 0.436f, &sh))
                return bgrx((int)(50 * sh), (int)(50 * sh), (int)(255 * sh));
            return bgrx(0, 0, 0);
        }
    }
    // ---- scrolling terminal (2 px per frame at 60 fps)
    {
        const int x0 = (int)(W * 0.04f), y0 = (int)(H * 0.10f);
        const int ww = (int)(W * 0.42f), wh = (int)(H * 0.38f);
        if (gx >= x0 && gx < x0 + ww && gy >= y0 && gy < y0 + wh) {
            if (gy - y0 < 12) return bgrx(60, 60, 70);
            const int scroll = (int)(p.t * 120.f);
            const int ty = gy - y0 - 12 + scroll, tx = gx - x0 - 4;
            const int row = ty / 16, col = tx / 8;
            const int len = (int)(hash3(row, 7, 1) % 70u);
            if (tx >= 0 && col < len) {
                const int px = tx % 8, py = ty % 16;
                if (px < 5 && py >= 4 && py < 13) {
                    const uint32_t glyph = hash3(row, col, 3);
                    const int bitidx = (py - 4) * 5 + px;
                    if ((glyph >> (bitidx % 32)) & 1) return bgrx(80, 230, 100);
                }
            }
            return bgrx(16, 20, 24);
        }
    }
    // ---- animated noise panel
    if (p.noise) {
        const int x0 = (int)(W * 0.04f), y0 = (int)(H * 0.55f);
        const int ww = (int)(W * 0.16f), wh = (int)(H * 0.22f);
        if (gx >= x0 && gx < x0 + ww && gy >= y0 && gy < y0 + wh) {
            const uint32_t h = hash3(gx, gy, p.frame_id * 2654435761u);
            const int v = h & 0xff;
            return bgrx(v, (h >> 8) & 0xff, v);
        }
    }
    return static_px(gx, gy, p);
}

// The parts of the desktop that never change (document window, taskbar, wallpaper): rendered
// once per session into a cache that the per-frame kernel copies wherever no animated element
// covers the pixel (the per-pixel wallpaper sinf was most of k_synth's 17 us at 1080p).
// noinline: one instance for both callers (k_synth_static and desktop_px), so the float
// wallpaper math cannot round differently under per-site FMA contraction.
__device__ __attribute__((noinline)) uint32_t static_px(int gx, int gy, const SynthParams& p) {
    const int W = p.wall_w, H = p.wall_h;
    // ---- static text window (document)
    {
        const int x0 = (int)(W * 0.25f), y0 = (int)(H * 0.52f);
        const int ww = (int)(W * 0.24f), wh = (int)(H * 0.36f);
        if (gx >= x0 && gx < x0 + ww && gy >= y0 && gy < y0 + wh) {
            if (gy - y0 < 12) return bgrx(60, 60, 70);
            const int ty = gy - y0 - 16, tx = gx - x0 - 8;
            const int row = ty / 14, col = tx / 7;
            const int len = 20 + (int)(hash3(row, 11, 5) % 30u);
            if (ty >= 0 && tx >= 0 && col < len && (ty % 14) >= 3 && (ty % 14) < 11 && (tx % 7) < 5 &&
                (hash3(row, col, 9) & 7) != 0 && ((hash3(row, col, 9) >> ((((ty % 14) - 3) * 5 + (tx % 7)) & 31)) & 1))
                return bgrx(20, 20, 20);
            return bgrx(250, 250, 248);
        }
    }
    // ---- taskbar
    if (gy >= H - 32) {
        const int slot = gx / 40;
        if ((gx % 40) >= 6 && (gx % 40) < 34 && gy >= H - 28 && gy < H - 4 && slot < 12)
            return bgrx(80 + (int)(hash3(slot, 1, 1) % 120u), 80 + (int)(hash3(slot, 2, 1) % 120u),
                        120 + (int)(hash3(slot, 3, 1) % 120u));
        return bgrx(30, 32, 40);
    }
    // ---- wallpaper: smooth gradient + soft diagonal bands
    const float fx = (float)gx / W, fy = (float)gy / H;
    const float band = 0.5f + 0.5f * sinf((fx * 3.f + fy * 2.f) * 3.14159265f);
    return bgrx((int)(20 + 40 * fy + 20 * band), (int)(40 + 60 * fy + 10 * band), (int)(90 + 110 * (1.f - fy * 0.5f)));
}

// bg: the session's static-layer cache (same size / pitch / origin), or nullptr.
__device__ __forceinline__ void synth_body(uint8_t* __restrict__ out, const SynthParams& p,
                                           const uint8_t* __restrict__ bg) {
    const int x4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const int y = blockIdx.y * blockDim.y + threadIdx.y;
    if (y >= p.height || x4 >= p.width) return;
    uint32_t v[4];
    const int gx = p.origin_x + x4, gy = p.origin_y + y;
    if (bg != nullptr && x4 + 4 <= p.width && !in_dyn(dyn_boxes(p), gx, 4, gy)) {
        const uint4 c = *reinterpret_cast<const uint4*>(bg + (size_t)y * p.pitch + 4 * x4);
        v[0] = c.x; v[1] = c.y; v[2] = c.z; v[3] = c.w;
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = (x4 + k < p.width) ? desktop_px(gx + k, gy, p) : 0u;
    }
    uint32_t* row = reinterpret_cast<uint32_t*>(out + (size_t)y * p.pitch);
    if (x4 + 4 <= p.width) {
        *reinterpret_cast<uint4*>(row + x4) = make_uint4(v[0], v[1], v[2], v[3]);
    } else {
        for (int k = 0; k < 4 && x4 + k < p.width; ++k) row[x4 + k] = v[k];
    }
}

__global__ __launch_bounds__(256) void k_synth(uint8_t* __restrict__ out, SynthParams p, const uint8_t* __restrict__ bg) {
    synth_body(out, p, bg);
}

__global__ __launch_bounds__(256) void k_synth_static(uint8_t* __restrict__ out, SynthParams p) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y * blockDim.y + threadIdx.y;
    if (x >= p.width || y >= p.height) return;
    reinterpret_cast<uint32_t*>(out + (size_t)y * p.pitch)[x] = static_px(p.origin_x + x, p.origin_y + y, p);
}

// Graph-replay variant: per-frame parameters come from device memory (uploaded by a memcpy
// node of the same graph), so the captured kernel node never changes.
__global__ __launch_bounds__(256) void k_synth_dev(uint8_t* __restrict__ out, const SynthParams* __restrict__ pp,
                                                   const uint8_t* __restrict__ bg) {
    const SynthParams p = *pp;
    synth_body(out, p, bg);
}

// BT.709 limited-range integer coefficients (x256); each row sums to 220 / 0 / 0.
__device__ __forceinline__ int y709(int r, int g, int b) { return ((47 * r + 157 * g + 16 * b + 128) >> 8) + 16; }
__device__ __forceinline__ int u709(int r, int g, int b) { return ((-26 * r - 86 * g + 112 * b + 128) >> 8) + 128; }
__device__ __forceinline__ int v709(int r, int g, int b) { return ((112 * r - 102 * g - 10 * b + 128) >> 8) + 128; }

__global__ __launch_bounds__(256) void k_bgrx_to_nv12(const uint8_t* __restrict__ in, int in_pitch, int w, int h,
                                                      uint8_t* __restrict__ yp, uint8_t* __restrict__ uvp,
                                                      int out_pitch, int coded_w, int coded_h) {
    const int bx = blockIdx.x * blockDim.x + threadIdx.x;  // 4-pixel column group
    const int by = blockIdx.y * blockDim.y + threadIdx.y;  // 2-row group
    const int x = bx * 4, y = by * 2;
    if (x >= coded_w || y >= coded_h) return;
    uint32_t px[2][4];
    const bool interior = (x + 4 <= w) && (y + 2 <= h);
    if (interior) {
        const uint4 a = *reinterpret_cast<const uint4*>(in + (size_t)y * in_pitch + x * 4);
        const uint4 b = *reinterpret_cast<const uint4*>(in + (size_t)(y + 1) * in_pitch + x * 4);
        px[0][0] = a.x; px[0][1] = a.y; px[0][2] = a.z; px[0][3] = a.w;
        px[1][0] = b.x; px[1][1] = b.y; px[1][2] = b.z; px[1][3] = b.w;
    } else {
        for (int r = 0; r < 2; ++r)
            for (int k = 0; k < 4; ++k) {
                const int sx = min(x + k, w - 1), sy = min(y + r, h - 1);
                px[r][k] = *reinterpret_cast<const uint32_t*>(in + (size_t)sy * in_pitch + sx * 4);
            }
    }
    uint32_t yw[2] = {0, 0};
    int rs[2] = {0, 0}, gs[2] = {0, 0}, bs[2] = {0, 0};
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t v = px[r][k];
            const int B = v & 0xff, G = (v >> 8) & 0xff, R = (v >> 16) & 0xff;
            yw[r] |= (uint32_t)y709(R, G, B) << (8 * k);
            rs[k >> 1] += R;
            gs[k >> 1] += G;
            bs[k >> 1] += B;
        }
    *reinterpret_cast<uint32_t*>(yp + (size_t)y * out_pitch + x) = yw[0];
    *reinterpret_cast<uint32_t*>(yp + (size_t)(y + 1) * out_pitch + x) = yw[1];
    uint32_t uvw = 0;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int R = (rs[c] + 2) >> 2, G = (gs[c] + 2) >> 2, B = (bs[c] + 2) >> 2;
        uvw |= (uint32_t)u709(R, G, B) << (16 * c);
        uvw |= (uint32_t)v709(R, G, B) << (16 * c + 8);
    }
    *reinterpret_cast<uint32_t*>(uvp + (size_t)(y / 2) * out_pitch + x) = uvw;
}

// ---- fused Lanczos scale + CSC.  Output tile 64 x 16 luma pixels, 256 threads, each
// thread produces a 2x2 output block (4 Y + one UV pair).
constexpr int kTileW = 64, kTileH = 16;

__global__ __launch_bounds__(256) void k_scale_to_nv12(const uint8_t* __restrict__ in, int in_pitch, int in_w,
                                                       int in_h, LanczosTables t, uint8_t* __restrict__ yp,
                                                       uint8_t* __restrict__ uvp, int out_pitch, int coded_w,
                                                       int coded_h, int max_nc, int max_nr) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int ox0 = blockIdx.x * kTileW, oy0 = blockIdx.y * kTileH;
    const int tid = threadIdx.x;
    const int oxl = min(ox0 + kTileW - 1, t.out_w - 1), oyl = min(oy0 + kTileH - 1, t.out_h - 1);
    const int oxf = min(ox0, t.out_w - 1), oyf = min(oy0, t.out_h - 1);
    const int xlo = t.x0[oxf], xhi = t.x0[oxl] + t.taps_x - 1;
    const int ylo = t.y0[oyf], yhi = t.y0[oyl] + t.taps_y - 1;
    const int nc = xhi - xlo + 1, nr = yhi - ylo + 1;
    const int tx = t.taps_x, ty = t.taps_y;
    // LDS: input footprint [nr][max_nc] BGRx | horizontal result [nr][kTileW] x RGB float |
    //      this tile's filter weights [kTileW][tx] + [kTileH][ty] and first-tap offsets
    uint32_t* lin = reinterpret_cast<uint32_t*>(smem);
    float* hr = reinterpret_cast<float*>(smem + (((size_t)max_nr * max_nc * 4 + 15) & ~(size_t)15));
    float* hg = hr + max_nr * kTileW;
    float* hb = hg + max_nr * kTileW;
    float* wxs = hb + max_nr * kTileW;
    float* wys = wxs + kTileW * tx;
    int* bx = reinterpret_cast<int*>(wys + kTileH * ty);
    int* by = bx + kTileW;
    for (int i = tid; i < nr * nc; i += 256) {
        const int r = i / nc, c = i - r * nc;
        const int sy = min(max(ylo + r, 0), in_h - 1), sx = min(max(xlo + c, 0), in_w - 1);
        lin[r * max_nc + c] = *reinterpret_cast<const uint32_t*>(in + (size_t)sy * in_pitch + sx * 4);
    }
    for (int i = tid; i < kTileW * tx; i += 256) {
        const int c = i / tx, k = i - c * tx;
        wxs[i] = t.wx[(size_t)min(ox0 + c, t.out_w - 1) * tx + k];
    }
    for (int i = tid; i < kTileH * ty; i += 256) {
        const int r = i / ty, k = i - r * ty;
        wys[i] = t.wy[(size_t)min(oy0 + r, t.out_h - 1) * ty + k];
    }
    if (tid < kTileW) bx[tid] = t.x0[min(ox0 + tid, t.out_w - 1)] - xlo;
    if (tid < kTileH) by[tid] = t.y0[min(oy0 + tid, t.out_h - 1)] - ylo;
    __syncthreads();
    for (int i = tid; i < nr * kTileW; i += 256) {
        const int r = i / kTileW, c = i - r * kTileW;
        const uint32_t* src = lin + r * max_nc + bx[c];
        const float* w = wxs + c * tx;
        float R = 0.f, G = 0.f, B = 0.f;
        for (int k = 0; k < tx; ++k) {
            const uint32_t v = src[k];
            const float wk = w[k];
            B += wk * (float)(v & 0xff);
            G += wk * (float)((v >> 8) & 0xff);
            R += wk * (float)((v >> 16) & 0xff);
        }
        hr[r * kTileW + c] = R;
        hg[r * kTileW + c] = G;
        hb[r * kTileW + c] = B;
    }
    __syncthreads();
    const int lx = (tid & 31) * 2, ly = (tid >> 5) * 2;
    int Rq[2][2], Gq[2][2], Bq[2][2];
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
        const int base = by[ly + dy];
        const float* w = wys + (ly + dy) * ty;
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
            const int c = lx + dx;
            float R = 0.f, G = 0.f, B = 0.f;
            for (int k = 0; k < ty; ++k) {
                const float wk = w[k];
                const int o = (base + k) * kTileW + c;
                R += wk * hr[o];
                G += wk * hg[o];
                B += wk * hb[o];
            }
            Rq[dy][dx] = min(max((int)lrintf(R), 0), 255);
            Gq[dy][dx] = min(max((int)lrintf(G), 0), 255);
            Bq[dy][dx] = min(max((int)lrintf(B), 0), 255);
        }
    }
    const int x = ox0 + lx, y = oy0 + ly;
    if (x >= coded_w || y >= coded_h) return;
    // output pixels beyond out_w/out_h replicate the last column/row (coded padding)
    for (int dy = 0; dy < 2; ++dy) {
        const int srcdy = (y + dy < t.out_h) ? dy : 0;
        uint16_t pair = 0;
        for (int dx = 0; dx < 2; ++dx) {
            const int srcdx = (x + dx < t.out_w) ? dx : 0;
            pair |= (uint16_t)(y709(Rq[srcdy][srcdx], Gq[srcdy][srcdx], Bq[srcdy][srcdx]) << (8 * dx));
        }
        *reinterpret_cast<uint16_t*>(yp + (size_t)(y + dy) * out_pitch + x) = pair;
    }
    const int R = (Rq[0][0] + Rq[0][1] + Rq[1][0] + Rq[1][1] + 2) >> 2;
    const int G = (Gq[0][0] + Gq[0][1] + Gq[1][0] + Gq[1][1] + 2) >> 2;
    const int B = (Bq[0][0] + Bq[0][1] + Bq[1][0] + Bq[1][1] + 2) >> 2;
    uvp[(size_t)(y / 2) * out_pitch + x] = (uint8_t)u709(R, G, B);
    uvp[(size_t)(y / 2) * out_pitch + x + 1] = (uint8_t)v709(R, G, B);
}

__global__ __launch_bounds__(256) void k_composite(const uint8_t* __restrict__ tile, int tile_pitch, int tw, int th,
                                                   uint8_t* __restrict__ dst, int dst_pitch, int dx, int dy) {
    const int x = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const int y = blockIdx.y;
    if (y >= th || x >= tw) return;
    const uint32_t* s = reinterpret_cast<const uint32_t*>(tile + (size_t)y * tile_pitch) + x;
    uint32_t* d = reinterpret_cast<uint32_t*>(dst + (size_t)(y + dy) * dst_pitch) + dx + x;
    if (x + 4 <= tw && ((dx & 3) == 0)) {
        *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(s);
    } else {
        for (int k = 0; k < 4 && x + k < tw; ++k) d[k] = s[k];
    }
}

// Tiled-wall composite of packed NV12 tiles (Y rows then interleaved UV rows, tile_w pitch,
// tiles in rank order) into the wall's Y / UV planes: one launch for every tile and both
// planes (blockIdx.z = tile, blockIdx.y = tile row incl. the UV rows), 16-byte copies.
__global__ __launch_bounds__(256) void k_composite_nv12(const uint8_t* __restrict__ tiles, int tw, int th, int cols,
                                                        uint8_t* __restrict__ y, uint8_t* __restrict__ uv, int pitch) {
    const int tile = blockIdx.z, row = blockIdx.y;
    const int x = (blockIdx.x * blockDim.x + threadIdx.x) * 16;
    if (x >= tw) return;
    const int ox = (tile % cols) * tw, oy = (tile / cols) * th;
    const uint8_t* src = tiles + (size_t)tile * tw * th * 3 / 2 + (size_t)row * tw + x;
    uint8_t* dst = row < th ? y + (size_t)(oy + row) * pitch + ox + x
                            : uv + (size_t)(oy / 2 + row - th) * pitch + ox + x;
    if (x + 16 <= tw && ((tw | pitch) & 15) == 0) {
        *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
    } else {
        for (int k = 0; k < 16 && x + k < tw; ++k) dst[k] = src[k];
    }
}

// One 256-thread workgroup per 8 rows; every thread owns 4-pixel dword columns (16-byte
// loads where aligned), one atomic per workgroup.
// Single-pass masked luma SSE: 16-byte loads, one partial per workgroup, the last workgroup
// to finish (device-scope counter) reduces the partials and stores the total straight into
// mapped pinned host memory -- one dispatch, no memset / D2H copy nodes on the stream.
// (The first version, 135 workgroups of 8 rows with an atomic into device memory plus a
// memset and a D2H copy, cost ~19 us per 1080p frame on the analysis stream: profiles/r02_b.)
__global__ __launch_bounds__(256) void k_sse_masked(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b,
                                                    int pitch, int w, int h, int rows, int mx0, int my0, int mx1,
                                                    int my1, unsigned long long* __restrict__ part,
                                                    unsigned int* __restrict__ counter,
                                                    unsigned long long* __restrict__ host_out) {
    const int nq = (w + 15) >> 4;
    const int y0 = blockIdx.x * rows;
    unsigned long long s = 0;
    for (int i = threadIdx.x; i < rows * nq; i += 256) {
        const int r = i / nq, x = (i - r * nq) * 16, y = y0 + r;
        if (y >= h) break;
        const uint4 va = *reinterpret_cast<const uint4*>(a + (size_t)y * pitch + x);
        const uint4 vb = *reinterpret_cast<const uint4*>(b + (size_t)y * pitch + x);
        const bool in_y = y >= my0 && y < my1;
        const uint32_t wa[4] = {va.x, va.y, va.z, va.w}, wb[4] = {vb.x, vb.y, vb.z, vb.w};
        uint32_t t = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int xx = x + k;
            const int d = (int)((wa[k >> 2] >> (8 * (k & 3))) & 0xff) - (int)((wb[k >> 2] >> (8 * (k & 3))) & 0xff);
            const bool masked = in_y && xx >= mx0 && xx < mx1;
            t += (xx < w && !masked) ? (uint32_t)(d * d) : 0u;  // <= 16 * 65025: no overflow
        }
        s += t;
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    __shared__ unsigned long long wpart[4];
    __shared__ bool last;
    if ((threadIdx.x & 63) == 0) wpart[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        part[blockIdx.x] = wpart[0] + wpart[1] + wpart[2] + wpart[3];
        __threadfence();
        last = atomicAdd(counter, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    unsigned long long t = 0;
    for (int i = threadIdx.x; i < (int)gridDim.x; i += 256) t += __atomic_load_n(part + i, __ATOMIC_RELAXED);
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    if ((threadIdx.x & 63) == 0) wpart[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        *host_out = wpart[0] + wpart[1] + wpart[2] + wpart[3];
        *counter = 0;  // ready for the next frame (stream-ordered)
    }
}

}  // namespace

int sse_masked_blocks(int w, int h) {
    const int nq = (w + 15) >> 4;
    const int rows = nq >= 256 ? 1 : 256 / nq;
    return (h + rows - 1) / rows;
}

void launch_sse_masked(const uint8_t* a, const uint8_t* b, int pitch, int w, int h, int mx0, int my0, int mx1,
                       int my1, unsigned long long* part, unsigned int* counter, unsigned long long* host_out,
                       hipStream_t stream) {
    if ((pitch & 15) != 0 || pitch < ((w + 15) & ~15) || (reinterpret_cast<uintptr_t>(a) & 15) ||
        (reinterpret_cast<uintptr_t>(b) & 15))
        throw std::invalid_argument("sse_masked: planes and pitch must be 16-byte aligned, pitch >= width");
    const int nq = (w + 15) >> 4;
    const int rows = nq >= 256 ? 1 : 256 / nq;
    hipLaunchKernelGGL(k_sse_masked, dim3(sse_masked_blocks(w, h)), dim3(256), 0, stream, a, b, pitch, w, h, rows,
                       mx0, my0, mx1, my1, part, counter, host_out);
}

void launch_synth(uint8_t* bgrx, const SynthParams& p, hipStream_t stream, const uint8_t* static_bg) {
    if (static_bg != nullptr && ((p.pitch & 15) || (reinterpret_cast<uintptr_t>(static_bg) & 15)))
        throw std::invalid_argument("synth: the static-layer cache needs a 16-byte aligned pitch");
    dim3 block(64, 4);
    dim3 grid((p.width / 4 + 63) / 64 + 1, (p.height + 3) / 4);
    hipLaunchKernelGGL(k_synth, grid, block, 0, stream, bgrx, p, static_bg);
}

void launch_synth_static(uint8_t* bgrx, const SynthParams& p, hipStream_t stream) {
    dim3 block(64, 4);
    dim3 grid((p.width + 63) / 64, (p.height + 3) / 4);
    hipLaunchKernelGGL(k_synth_static, grid, block, 0, stream, bgrx, p);
}

void launch_synth_dev(uint8_t* bgrx, const SynthParams* d_params, int width, int height, hipStream_t stream,
                      const uint8_t* static_bg) {
    dim3 block(64, 4);
    dim3 grid((width / 4 + 63) / 64 + 1, (height + 3) / 4);
    hipLaunchKernelGGL(k_synth_dev, grid, block, 0, stream, bgrx, d_params, static_bg);
}

void launch_bgrx_to_nv12(const uint8_t* bgrx, int in_pitch, int w, int h, uint8_t* y, uint8_t* uv, int out_pitch,
                         int coded_w, int coded_h, hipStream_t stream) {
    dim3 block(64, 4);
    dim3 grid((coded_w / 4 + 63) / 64, (coded_h / 2 + 3) / 4);
    hipLaunchKernelGGL(k_bgrx_to_nv12, grid, block, 0, stream, bgrx, in_pitch, w, h, y, uv, out_pitch, coded_w,
                       coded_h);
}

void launch_scale_to_nv12(const uint8_t* bgrx, int in_pitch, int in_w, int in_h, const LanczosTables& t, uint8_t* y,
                          uint8_t* uv, int out_pitch, int coded_w, int coded_h, hipStream_t stream) {
    // worst-case footprint of a tile: scale * tile + taps
    const float sx = (float)in_w / t.out_w, sy = (float)in_h / t.out_h;
    const int max_nc = (int)ceilf(sx * kTileW) + t.taps_x + 2;
    const int max_nr = (int)ceilf(sy * kTileH) + t.taps_y + 2;
    const size_t lds = (((size_t)max_nr * max_nc * 4 + 15) & ~(size_t)15) + (size_t)max_nr * kTileW * 12 +
                       (size_t)(kTileW * t.taps_x + kTileH * t.taps_y) * 4 + (kTileW + kTileH) * 4;
    if (lds > 160 * 1024) throw std::runtime_error("scale_to_nv12: scale factor too large for one LDS tile");
    if (lds > 64 * 1024) {
        static bool raised = false;
        if (!raised) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scale_to_nv12),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            raised = true;
        }
    }
    dim3 grid((coded_w + kTileW - 1) / kTileW, (coded_h + kTileH - 1) / kTileH);
    hipLaunchKernelGGL(k_scale_to_nv12, grid, dim3(256), lds, stream, bgrx, in_pitch, in_w, in_h, t, y, uv, out_pitch,
                       coded_w, coded_h, max_nc, max_nr);
}

void launch_composite(const uint8_t* tile, int tile_pitch, int tw, int th, uint8_t* dst, int dst_pitch, int dx, int dy,
                      hipStream_t stream) {
    dim3 grid((tw / 4 + 255) / 256 + 1, th);
    hipLaunchKernelGGL(k_composite, grid, dim3(256), 0, stream, tile, tile_pitch, tw, th, dst, dst_pitch, dx, dy);
}

void launch_composite_nv12(const uint8_t* tiles, int tw, int th, int cols, int rows, uint8_t* y, uint8_t* uv,
                           int pitch, hipStream_t stream) {
    if ((tw & 1) || (th & 1) || pitch < cols * tw) throw std::invalid_argument("composite_nv12: bad tile geometry");
    dim3 grid((tw / 16 + 255) / 256 + 1, th + th / 2, cols * rows);
    hipLaunchKernelGGL(k_composite_nv12, grid, dim3(256), 0, stream, tiles, tw, th, cols, y, uv, pitch);
}

}  // namespace pix
}  // namespace mx
