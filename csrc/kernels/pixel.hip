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

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <type_traits>

#include "pixel.h"
#include "../common/hip_check.h"

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

// Frame start stamp: the first thread of the grid stores the device wall clock.
__device__ __forceinline__ void stamp_start(uint64_t* ts) {
    if (ts && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && threadIdx.y == 0) *ts = wall_clock64();
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
__device__ __forceinline__ DynBoxes dyn_boxes(const SynthParams& p, int wx, int wy, int mw, int mh) {
    const int W = p.wall_w, H = p.wall_h;
    DynBoxes b;
    b.x0[0] = kBarX - kBarCell; b.y0[0] = kBarY - kBarCell;
    b.x1[0] = kBarX + 33 * kBarCell; b.y1[0] = kBarY + 3 * kBarCell;
    b.x0[1] = p.cursor_x >= 0 ? p.cursor_x : 0; b.y0[1] = p.cursor_y;
    b.x1[1] = p.cursor_x >= 0 ? p.cursor_x + 12 : 0; b.y1[1] = p.cursor_y + 19;
    b.x0[2] = wx; b.y0[2] = wy;  // the moving window, from the same per-frame constants desktop_px uses
    b.x1[2] = b.x0[2] + mw; b.y1[2] = b.y0[2] + mh;
    b.x0[3] = (int)(W * 0.55f); b.y0[3] = (int)(H * 0.10f);
    b.x1[3] = b.x0[3] + (int)(W * 0.38f); b.y1[3] = b.y0[3] + (int)(H * 0.50f);
    b.x0[4] = (int)(W * 0.04f); b.y0[4] = (int)(H * 0.10f);
    b.x1[4] = b.x0[4] + (int)(W * 0.42f); b.y1[4] = b.y0[4] + (int)(H * 0.38f);
    b.x0[5] = (int)(W * 0.04f); b.y0[5] = (int)(H * 0.55f);
    b.x1[5] = p.noise ? b.x0[5] + (int)(W * 0.16f) : b.x0[5]; b.y1[5] = b.y0[5] + (int)(H * 0.22f);
    return b;
}
// Whether any of pixels [gx, gx+n) of row gy lies in an animated element's bounds (2-pixel
// margin kept from when the window position was computed twice under different FMA contraction).
__device__ __forceinline__ bool in_dyn(const DynBoxes& b, int gx, int n, int gy) {
    bool hit = false;
#pragma unroll
    for (int k = 0; k < 6; ++k)
        hit |= b.x1[k] > b.x0[k] && gy >= b.y0[k] - 2 && gy < b.y1[k] + 2 && gx + n > b.x0[k] - 2 && gx < b.x1[k] + 2;
    return hit;
}

// Per-frame constants of the animated elements, formed once per thread (the per-pixel sinf of
// the moving window's path and the gear angles were most of k_synth's VALU work)
struct FrameConsts {
    int wx, wy, mw, mh;       // moving window
    float gear_a[3];          // gear rotation angles
};
__device__ __forceinline__ FrameConsts frame_consts(const SynthParams& p) {
    const int W = p.wall_w, H = p.wall_h;
    FrameConsts f;
    f.mw = W / 8 > 48 ? W / 8 : 48;
    f.mh = H / 8 > 32 ? H / 8 : 32;
    const float cxm = W * 0.5f, cym = H * 0.62f;
    f.wx = (int)(cxm + W * 0.18f * sinf(p.t * 0.7f)) - f.mw / 2;
    f.wy = (int)(cym + H * 0.12f * sinf(p.t * 1.1f)) - f.mh / 2;
    const float a = p.t * 1.5707963f;  // 90 deg/s like glxgears' default speed order
    f.gear_a[0] = a;
    f.gear_a[1] = -2.f * a - 0.157f;
    f.gear_a[2] = -2.f * a - 0.436f;
    return f;
}

// ---- motion content (SynthParams::content 1)
__device__ __forceinline__ bool in_barcode(int gx, int gy) {
    return gy >= kBarY - kBarCell && gy < kBarY + 3 * kBarCell && gx >= kBarX - kBarCell && gx < kBarX + 33 * kBarCell;
}
__device__ __forceinline__ void video_rect(const SynthParams& p, int* x0, int* y0, int* x1, int* y1) {
    *x0 = (int)(p.wall_w * kVideoX);
    *y0 = (int)(p.wall_h * kVideoY);
    *x1 = *x0 + (int)(p.wall_w * kVideoW);
    *y1 = *y0 + (int)(p.wall_h * kVideoH);
}
// pan offset of frame time t: 3 px / frame right, 1 px / frame down at 60 fps (integer, wrapping)
__device__ __forceinline__ void pan_of(const SynthParams& p, int* px, int* py) {
    const int f = (int)(p.t * 60.f + 0.5f);
    *px = (3 * f) % p.wall_w;
    *py = f % p.wall_h;
}
// sub-sample pan of frame time t (content 2), in quarter samples: 2.5 px / frame right, 0.75 px /
// frame down at 60 fps, so consecutive frames differ by fractional displacements (qpel motion
// search, the six-tap / eight-tap interpolation and the deblocking decision all get exercised)
__device__ __forceinline__ void pan_q4(const SynthParams& p, int* qx, int* qy) {
    const int f = (int)(p.t * 60.f + 0.5f);
    *qx = (10 * f) % (4 * p.wall_w);
    *qy = (3 * f) % (4 * p.wall_h);
}
// smooth value noise: bilinear, smoothstep-weighted interpolation of a hashed integer lattice
__device__ __forceinline__ float vnoise(float x, float y, uint32_t seed) {
    const float fx = floorf(x), fy = floorf(y);
    const int ix = (int)fx, iy = (int)fy;
    float u = x - fx, v = y - fy;
    u = u * u * (3.f - 2.f * u);
    v = v * v * (3.f - 2.f * v);
    const float a = (float)(hash3((uint32_t)ix, (uint32_t)iy, seed) & 1023u);
    const float b = (float)(hash3((uint32_t)ix + 1u, (uint32_t)iy, seed) & 1023u);
    const float c = (float)(hash3((uint32_t)ix, (uint32_t)iy + 1u, seed) & 1023u);
    const float d = (float)(hash3((uint32_t)ix + 1u, (uint32_t)iy + 1u, seed) & 1023u);
    return ((a + (b - a) * u) + ((c + (d - c) * u) - (a + (b - a) * u)) * v) * (1.f / 1023.f);
}
// video-like texture at panel coordinates (u, v): three octaves of value noise drifting at
// different speeds (so the motion is not one translation), mapped through phase-shifted colour
// waves that also cycle slowly
__device__ uint32_t video_pxf(float u, float v, float t) {
    const float x = u * (1.f / 96.f), y = v * (1.f / 96.f);
    const float n = 0.55f * vnoise(x + 0.35f * t, y + 0.12f * t, 11u) +
                    0.30f * vnoise(2.1f * x - 0.6f * t, 2.1f * y + 0.25f * t, 23u) +
                    0.15f * vnoise(4.3f * x + 0.9f * t, 4.3f * y - 0.7f * t, 37u);
    const float ph = 6.2831853f * n;
    const int r = (int)(128.f + 100.f * __sinf(ph + 0.4f * t));
    const int g = (int)(128.f + 90.f * __sinf(1.3f * ph + 2.1f));
    const int b = (int)(128.f + 100.f * __sinf(0.8f * ph + 4.2f - 0.3f * t));
    return bgrx(r, g, b);
}
__device__ __forceinline__ uint32_t video_px(int u, int v, float t) { return video_pxf((float)u, (float)v, t); }

__device__ uint32_t desktop_px(int gx, int gy, const SynthParams& p, const FrameConsts& fc) {
    const int W = p.wall_w, H = p.wall_h;
    // ---- barcode (frame id + timestamp), always on top
    if (p.content == 0 && gy >= kBarY - kBarCell && gy < kBarY + 2 * kBarCell + kBarCell && gx >= kBarX - kBarCell &&
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
        const int mw = fc.mw, mh = fc.mh, wx = fc.wx, wy = fc.wy;
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
            float sh;
            if (gear_hit(sx + 3.0f, sy + 2.0f, 1.0f, 4.0f, 0.7f, 20, fc.gear_a[0], &sh))
                return bgrx((int)(204 * sh), (int)(25 * sh), 0);
            if (gear_hit(sx - 3.1f, sy + 2.0f, 0.5f, 2.0f, 0.7f, 10, fc.gear_a[1], &sh))
                return bgrx(0, (int)(204 * sh), (int)(50 * sh));
            if (gear_hit(sx + 3.1f, sy - 4.2f, 1.3f, 2.0f, 0.7f, 10, fc.gear_a[2], &sh))
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

// barcode pixel (frame id + timestamp) at screen coordinates inside in_barcode()
__device__ __forceinline__ uint32_t barcode_px(int gx, int gy, const SynthParams& p) {
    const int cx = (gx - kBarX), cy = (gy - kBarY);
    if (cx < 0 || cy < 0 || cx >= 32 * kBarCell || cy >= 2 * kBarCell) return bgrx(96, 96, 96);  // quiet zone
    const int bit = 31 - cx / kBarCell;
    const uint32_t word = (cy / kBarCell) == 0 ? p.frame_id : p.timestamp_us;
    const int v = ((word >> bit) & 1) ? 255 : 0;
    return bgrx(v, v, v);
}

// Motion content: screen pixel (gx, gy) -- barcode and video panel screen-fixed, the rest the
// panned desktop (static layer from the cache when given).
__device__ __forceinline__ uint32_t motion_px(int gx, int gy, const SynthParams& p, const FrameConsts& fc,
                                              const uint8_t* __restrict__ bg, int px, int py, int vx0, int vy0,
                                              int vx1, int vy1, const DynBoxes& boxes) {
    if (in_barcode(gx, gy)) return barcode_px(gx, gy, p);
    if (gx >= vx0 && gx < vx1 && gy >= vy0 && gy < vy1) return video_px(gx - vx0, gy - vy0, p.t);
    int dx = gx + px, dy = gy + py;
    dx -= dx >= p.wall_w ? p.wall_w : 0;
    dy -= dy >= p.wall_h ? p.wall_h : 0;
    if (bg != nullptr && p.origin_x == 0 && p.origin_y == 0 && !in_dyn(boxes, dx, 1, dy))
        return *reinterpret_cast<const uint32_t*>(bg + (size_t)dy * p.pitch + 4 * dx);
    return desktop_px(dx, dy, p, fc);
}

// Sub-sample motion content (content 2): the desktop pans by a fractional displacement (pan_q4),
// sampled bilinearly from the four covering desktop pixels (quarter-sample weights, per channel),
// and the video panel's texture zooms continuously (scale 0.8 .. 1.1 over ~12 s) -- a scaled video.
__device__ __forceinline__ uint32_t desk_at(int dx, int dy, const SynthParams& p, const FrameConsts& fc,
                                            const uint8_t* __restrict__ bg, const DynBoxes& boxes) {
    dx -= dx >= p.wall_w ? p.wall_w : 0;
    dy -= dy >= p.wall_h ? p.wall_h : 0;
    if (bg != nullptr && p.origin_x == 0 && p.origin_y == 0 && !in_dyn(boxes, dx, 1, dy))
        return *reinterpret_cast<const uint32_t*>(bg + (size_t)dy * p.pitch + 4 * dx);
    return desktop_px(dx, dy, p, fc);
}
__device__ __forceinline__ uint32_t subpel_px(int gx, int gy, const SynthParams& p, const FrameConsts& fc,
                                              const uint8_t* __restrict__ bg, int qx, int qy, int vx0, int vy0,
                                              int vx1, int vy1, const DynBoxes& boxes) {
    if (in_barcode(gx, gy)) return barcode_px(gx, gy, p);
    if (gx >= vx0 && gx < vx1 && gy >= vy0 && gy < vy1) {
        const float s = 0.95f + 0.15f * __sinf(0.5f * p.t);
        const float cu = 0.5f * (vx1 - vx0), cv = 0.5f * (vy1 - vy0);
        return video_pxf(cu + ((float)(gx - vx0) - cu) * s, cv + ((float)(gy - vy0) - cv) * s, p.t);
    }
    const int ix = gx + (qx >> 2), iy = gy + (qy >> 2), fx = qx & 3, fy = qy & 3;
    const uint32_t a = desk_at(ix, iy, p, fc, bg, boxes);
    if ((fx | fy) == 0) return a;
    const uint32_t b = desk_at(ix + 1, iy, p, fc, bg, boxes), c = desk_at(ix, iy + 1, p, fc, bg, boxes),
                   d = desk_at(ix + 1, iy + 1, p, fc, bg, boxes);
    const int wa = (4 - fx) * (4 - fy), wb = fx * (4 - fy), wc = (4 - fx) * fy, wd = fx * fy;
    uint32_t out = 0;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        const int sh = 8 * ch;
        const int v = (wa * (int)((a >> sh) & 0xff) + wb * (int)((b >> sh) & 0xff) + wc * (int)((c >> sh) & 0xff) +
                       wd * (int)((d >> sh) & 0xff) + 8) >> 4;
        out |= (uint32_t)v << sh;
    }
    return out;
}

// bg: the session's static-layer cache (same size / pitch / origin), or nullptr.
__device__ __forceinline__ void synth_body(uint8_t* __restrict__ out, const SynthParams& p,
                                           const uint8_t* __restrict__ bg) {
    stamp_start(p.ts);
    const int x4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const int y = blockIdx.y * blockDim.y + threadIdx.y;
    if (y >= p.height || x4 >= p.width) return;
    uint32_t v[4];
    const int gx = p.origin_x + x4, gy = p.origin_y + y;
    const FrameConsts fc = frame_consts(p);
    if (p.content == 1 || p.content == 2) {
        int px, py, vx0, vy0, vx1, vy1;
        if (p.content == 1)
            pan_of(p, &px, &py);
        else
            pan_q4(p, &px, &py);
        video_rect(p, &vx0, &vy0, &vx1, &vy1);
        const DynBoxes boxes = dyn_boxes(p, fc.wx, fc.wy, fc.mw, fc.mh);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            v[k] = (x4 + k >= p.width) ? 0u
                   : p.content == 1 ? motion_px(gx + k, gy, p, fc, bg, px, py, vx0, vy0, vx1, vy1, boxes)
                                    : subpel_px(gx + k, gy, p, fc, bg, px, py, vx0, vy0, vx1, vy1, boxes);
        uint32_t* row = reinterpret_cast<uint32_t*>(out + (size_t)y * p.pitch);
        if (x4 + 4 <= p.width)
            *reinterpret_cast<uint4*>(row + x4) = make_uint4(v[0], v[1], v[2], v[3]);
        else
            for (int k = 0; k < 4 && x4 + k < p.width; ++k) row[x4 + k] = v[k];
        return;
    }
    if (bg != nullptr && x4 + 4 <= p.width && !in_dyn(dyn_boxes(p, fc.wx, fc.wy, fc.mw, fc.mh), gx, 4, gy)) {
        const uint4 c = *reinterpret_cast<const uint4*>(bg + (size_t)y * p.pitch + 4 * x4);
        v[0] = c.x; v[1] = c.y; v[2] = c.z; v[3] = c.w;
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = (x4 + k < p.width) ? desktop_px(gx + k, gy, p, fc) : 0u;
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
                                                      int out_pitch, int coded_w, int coded_h, uint64_t* ts) {
    stamp_start(ts);
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
//  * the input footprint is staged into LDS with 16-byte loads from a 4-pixel aligned start
//    (clamped per pixel only at picture borders);
//  * the horizontal pass keeps its result as int16 fixed point (x16, 6 B per pixel instead of
//    12 B of float RGB), so a 4K->1080p tile needs ~42 KB of LDS instead of ~62 KB and three
//    workgroups fit a CU;
//  * the UV pair of a 2x2 block is one 16-bit store.
// (The first version -- 4-byte footprint loads, float RGB intermediate, byte UV stores -- is
// measured in profiles/r02_scale.)
constexpr int kTileW = 64, kTileH = 16;
constexpr float kHFix = 16.f;  // horizontal-pass fixed-point scale

__global__ __launch_bounds__(256) void k_scale_to_nv12(const uint8_t* __restrict__ in, int in_pitch, int in_w,
                                                       int in_h, LanczosTables t, uint8_t* __restrict__ yp,
                                                       uint8_t* __restrict__ uvp, int out_pitch, int coded_w,
                                                       int coded_h, int max_nc, int max_nr, int vec, uint64_t* ts) {
    stamp_start(ts);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int ox0 = blockIdx.x * kTileW, oy0 = blockIdx.y * kTileH;
    const int tid = threadIdx.x;
    const int oxl = min(ox0 + kTileW - 1, t.out_w - 1), oyl = min(oy0 + kTileH - 1, t.out_h - 1);
    const int oxf = min(ox0, t.out_w - 1), oyf = min(oy0, t.out_h - 1);
    const int xlo = t.x0[oxf] & ~3, xhi = t.x0[oxl] + t.taps_x - 1;  // 4-pixel aligned footprint start
    const int ylo = t.y0[oyf], yhi = t.y0[oyl] + t.taps_y - 1;
    const int nq = (xhi - xlo + 4) >> 2, nr = yhi - ylo + 1;  // footprint: nq pixel quads x nr rows
    const int tx = t.taps_x, ty = t.taps_y;
    // LDS: footprint [nr][max_nc] BGRx | horizontal result [3][nr][kTileW] int16 |
    //      this tile's filter weights [kTileW][tx] + [kTileH][ty] and first-tap offsets
    uint32_t* lin = reinterpret_cast<uint32_t*>(smem);
    int16_t* hrgb = reinterpret_cast<int16_t*>(smem + (((size_t)max_nr * max_nc * 4 + 15) & ~(size_t)15));
    float* wxs = reinterpret_cast<float*>(hrgb + ((3 * max_nr * kTileW + 7) & ~7));
    float* wys = wxs + kTileW * tx;
    int* bx = reinterpret_cast<int*>(wys + kTileH * ty);
    int* by = bx + kTileW;
    for (int i = tid; i < nr * nq; i += 256) {
        const int r = i / nq, q = i - r * nq;
        const int sy = min(max(ylo + r, 0), in_h - 1), sx = xlo + 4 * q;
        const uint8_t* row = in + (size_t)sy * in_pitch;
        uint4 v;
        if (vec && sx >= 0 && sx + 4 <= in_w) {  // (vec: 16-byte aligned rows)
            v = *reinterpret_cast<const uint4*>(row + (size_t)sx * 4);
        } else {
            v.x = *reinterpret_cast<const uint32_t*>(row + (size_t)min(max(sx, 0), in_w - 1) * 4);
            v.y = *reinterpret_cast<const uint32_t*>(row + (size_t)min(max(sx + 1, 0), in_w - 1) * 4);
            v.z = *reinterpret_cast<const uint32_t*>(row + (size_t)min(max(sx + 2, 0), in_w - 1) * 4);
            v.w = *reinterpret_cast<const uint32_t*>(row + (size_t)min(max(sx + 3, 0), in_w - 1) * 4);
        }
        *reinterpret_cast<uint4*>(lin + r * max_nc + 4 * q) = v;
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
    // horizontal pass: a thread keeps one output column (tid % 64) for all its rows, so that
    // column's taps / weights stay in registers; R and G accumulate as a packed float pair
    // (v_pk_fma_f32), B on its own.  Result: int16 fixed point, R|G packed in one dword
    // plane and B in another, so the vertical pass reads two adjacent columns per load.
    typedef float f2 __attribute__((ext_vector_type(2)));
    const int hplane = max_nr * kTileW;
    uint32_t* hrg = reinterpret_cast<uint32_t*>(hrgb);  // [nr][kTileW] (R | G << 16)
    int16_t* hb = hrgb + 2 * hplane;                     // [nr][kTileW]
    {
        const int c = tid & (kTileW - 1);
        constexpr int kRegTaps = 20;
        float wr[kRegTaps];
#pragma unroll
        for (int k = 0; k < kRegTaps; ++k) wr[k] = k < tx ? wxs[c * tx + k] : 0.f;
        const int c0 = bx[c];
        for (int r = tid >> 6; r < nr; r += 256 / kTileW) {
            const uint32_t* src = lin + r * max_nc + c0;
            f2 rg = {0.f, 0.f};
            float B = 0.f;
            if (tx <= kRegTaps) {
#pragma unroll
                for (int k = 0; k < kRegTaps; ++k) {
                    if (k >= tx) break;
                    const uint32_t v = src[k];
                    const f2 p = {(float)((v >> 16) & 0xffu) /* R */, (float)((v >> 8) & 0xffu)};
                    rg = __builtin_elementwise_fma((f2){wr[k], wr[k]}, p, rg);
                    B = fmaf(wr[k], (float)((v >> 0) & 0xffu), B);
                }
            } else {  // very large scale factors: weights from LDS
                for (int k = 0; k < tx; ++k) {
                    const uint32_t v = src[k];
                    const float wk = wxs[c * tx + k];
                    const f2 p = {(float)((v >> 16) & 0xffu), (float)((v >> 8) & 0xffu)};
                    rg = __builtin_elementwise_fma((f2){wk, wk}, p, rg);
                    B = fmaf(wk, (float)((v >> 0) & 0xffu), B);
                }
            }
            const int R16 = (int)lrintf(rg.x * kHFix), G16 = (int)lrintf(rg.y * kHFix);
            hrg[r * kTileW + c] = (uint32_t)(R16 & 0xffff) | ((uint32_t)G16 << 16);
            hb[r * kTileW + c] = (int16_t)lrintf(B * kHFix);
        }
    }
    __syncthreads();
    // vertical pass: 2x2 outputs per thread; each tap reads R|G of both columns (two dwords)
    // and B of both columns (one dword)
    const int lx = (tid & 31) * 2, ly = (tid >> 5) * 2;
    int Rq[2][2], Gq[2][2], Bq[2][2];
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
        const int base = by[ly + dy];
        const float* w = wys + (ly + dy) * ty;
        f2 rg0 = {0.f, 0.f}, rg1 = {0.f, 0.f}, b01 = {0.f, 0.f};
        for (int k = 0; k < ty; ++k) {
            const float wk = w[k];
            const int o = (base + k) * kTileW + lx;
            const uint2 q = *reinterpret_cast<const uint2*>(hrg + o);       // columns lx, lx + 1
            const uint32_t bb = *reinterpret_cast<const uint32_t*>(hb + o);  // B of both columns
            const f2 p0 = {(float)(int16_t)(q.x & 0xffff), (float)(int16_t)(q.x >> 16)};
            const f2 p1 = {(float)(int16_t)(q.y & 0xffff), (float)(int16_t)(q.y >> 16)};
            const f2 pb = {(float)(int16_t)(bb & 0xffff), (float)(int16_t)(bb >> 16)};
            const f2 ww = {wk, wk};
            rg0 = __builtin_elementwise_fma(ww, p0, rg0);
            rg1 = __builtin_elementwise_fma(ww, p1, rg1);
            b01 = __builtin_elementwise_fma(ww, pb, b01);
        }
        const float inv = 1.f / kHFix;
        Rq[dy][0] = min(max((int)lrintf(rg0.x * inv), 0), 255);
        Gq[dy][0] = min(max((int)lrintf(rg0.y * inv), 0), 255);
        Rq[dy][1] = min(max((int)lrintf(rg1.x * inv), 0), 255);
        Gq[dy][1] = min(max((int)lrintf(rg1.y * inv), 0), 255);
        Bq[dy][0] = min(max((int)lrintf(b01.x * inv), 0), 255);
        Bq[dy][1] = min(max((int)lrintf(b01.y * inv), 0), 255);
    }
    const int x = ox0 + lx, y = oy0 + ly;
    if (x >= coded_w || y >= coded_h) return;
    // output pixels beyond out_w/out_h replicate the last column/row (coded padding)
    // (selects, not dynamic indices: keeps the 2x2 block in registers)
    if (y + 1 >= t.out_h) {
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) Rq[1][dx] = Rq[0][dx], Gq[1][dx] = Gq[0][dx], Bq[1][dx] = Bq[0][dx];
    }
    if (x + 1 >= t.out_w) {
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) Rq[dy][1] = Rq[dy][0], Gq[dy][1] = Gq[dy][0], Bq[dy][1] = Bq[dy][0];
    }
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
        const uint16_t pair = (uint16_t)(y709(Rq[dy][0], Gq[dy][0], Bq[dy][0]) |
                                         (y709(Rq[dy][1], Gq[dy][1], Bq[dy][1]) << 8));
        *reinterpret_cast<uint16_t*>(yp + (size_t)(y + dy) * out_pitch + x) = pair;
    }
    const int R = (Rq[0][0] + Rq[0][1] + Rq[1][0] + Rq[1][1] + 2) >> 2;
    const int G = (Gq[0][0] + Gq[0][1] + Gq[1][0] + Gq[1][1] + 2) >> 2;
    const int B = (Bq[0][0] + Bq[0][1] + Bq[1][0] + Bq[1][1] + 2) >> 2;
    *reinterpret_cast<uint16_t*>(uvp + (size_t)(y / 2) * out_pitch + x) =
        (uint16_t)(u709(R, G, B) | (v709(R, G, B) << 8));
}

// ---------------------------------------------------------------- MFMA Lanczos scaler
// Both resampling passes are banded matrix products, so they run on the matrix cores
// (v_mfma_f32_32x32x16_f16).  A workgroup (2 waves) owns a 64 x 32 output tile; each wave a
// 32 x 32 block.  Per 32-row block b of the input footprint and colour channel c:
//   X = In_c[rows of b][K window] * Wh[K window][32 output columns]      (horizontal)
//   Y_c += Wv[32 output rows][rows of b] * X                              (vertical)
// X's accumulator (output column on the lane, input rows in registers) is the vertical
// product's B operand as it stands (rows in the permuted k order of the fragment map; the
// host lays Wv's fragments out in that order), so X never goes through LDS.  Input pixels
// enter as f16 subnormals: v_perm puts one channel byte of two pixels in the low bytes of two
// halves (0x00pp = p * 2^-24, exact), one instruction per dword and no bias to remove.  The
// horizontal weights carry 2^14 and the vertical ones 2^10, so X = 2^-10 * (filtered row),
// a normal f16 with the precision of the former 1024 + p form, and Y is in pixel units.
// The footprint is staged global -> LDS with 16-byte LDS-DMA (global_load_lds_dwordx4); the
// weights of taps outside the picture are folded into its edge column, so only quads that
// straddle the right edge (input widths not a multiple of 4) are rewritten with clamped pixels.
constexpr float kMfHScale = 16384.f, kMfVScale = 1024.f;  // 2^14 * 2^10 * 2^-24 = 1
constexpr int kMfKs = 8;  // max horizontal K-steps (16 input columns each) per 32 output columns
// K-step counts k_scale_mfma is instantiated for: the smallest one >= n (n <= kMfKs)
constexpr int scale_mfma_nk(int n) { return n <= 2 ? 2 : n <= 6 ? n : 8; }
constexpr int kMfRb = 4;  // max 32-row input blocks per 32 output rows
constexpr int kStripRing = 3;  // k_scale_strip: LDS ring of 32-row input blocks (one computed, two in flight)
constexpr int kStripMaxT = 4;  // k_scale_strip: most 32-row output tiles per workgroup
typedef _Float16 mf_h8 __attribute__((ext_vector_type(8)));
typedef float mf_f16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void_t;

// Per-workgroup phase stamps of k_scale_mfma for tools/scale_stamps.hip (compiled out unless
// MX_SCALE_STAMPS is defined): [wg][0] = s_memrealtime at entry, [wg][1..6] = s_memtime at the
// phases named in mf_main / k_scale_mfma, [wg][7] = s_memrealtime at exit.
#ifdef MX_SCALE_STAMPS
__device__ uint64_t g_scale_stamps[4096 * 8];
#define MF_STAMP(k, v)                                                                                  \
    do {                                                                                                \
        if (threadIdx.x == 0) g_scale_stamps[(blockIdx.y * gridDim.x + blockIdx.x) * 8 + (k)] = (v);    \
    } while (0)
#else
#define MF_STAMP(k, v) \
    do {               \
    } while (0)
#endif

__device__ __forceinline__ mf_h8 mf_chan(const uint4& a, const uint4& b, uint32_t sel) {
    uint4 r;
    r.x = __builtin_amdgcn_perm(a.y, a.x, sel);
    r.y = __builtin_amdgcn_perm(a.w, a.z, sel);
    r.z = __builtin_amdgcn_perm(b.y, b.x, sel);
    r.w = __builtin_amdgcn_perm(b.w, b.z, sel);
    return __builtin_bit_cast(mf_h8, r);
}

__device__ __forceinline__ int clamp255(float v) { return min(max((int)__builtin_rintf(v), 0), 255); }

// Stage rows [r0, r0 + 32) of the footprint (clipped to nr) into `buf` with LDS-DMA, one
// footprint row per wave instruction (rows wave, wave + 2, ...: 16 instructions per wave for a
// full block): lane q < nq copies input pixels xlo + 4q .. +3 (its clamped byte offset `loff`)
// of input row ylo + r0 + r to LDS quad r * nq + q.
// Through a buffer resource over the picture: the lane's byte offset in the vector offset and
// the row's in the scalar offset, so a row costs no per-lane address arithmetic.
__device__ __forceinline__ void mf_stage(const uint8_t* __restrict__ in, int in_pitch, int in_h, int ylo, int r0,
                                         int nr, int nq, uint32_t loff, char* buf, int wave, int lane) {
    const int rows = min(32, nr - r0);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(in), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int r = wave + 2 * i;
        const int sy = min(max(ylo + r0 + r, 0), in_h - 1);
        if (r < rows && lane < nq)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(buf + (size_t)r * nq * 16), 16, (int)loff,
                                                     sy * in_pitch, 0, 0);
    }
}

// DMA instructions mf_stage issues for the block at row r0 (wave-uniform).
__device__ __forceinline__ int mf_stage_count(int r0, int nr, int wave) {
    const int rows = min(32, nr - r0);
    return rows > wave ? (rows - wave + 1) >> 1 : 0;
}

// s_waitcnt vmcnt(n) for a wave-uniform n in 0..16 (the immediate must be a constant)
template <int N = 16>
__device__ __forceinline__ void wait_vm_le(int n) {
    if constexpr (N == 0) {
        __builtin_amdgcn_s_waitcnt(0x0F70);
    } else {
        if (n >= N) {
            __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 15) | ((N >> 4) << 14));
            return;
        }
        wait_vm_le<N - 1>(n);
    }
}

// Workgroup barrier that leaves LDS-DMA in flight: __syncthreads() makes hipcc drain vmcnt
// to 0 first; the waits that matter here are explicit (LDS accesses: lgkmcnt(0)).
__device__ __forceinline__ void mf_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
}

// Quads crossing the left / right image edge, after their block's DMA landed: the DMA read the
// clamped quad (pixels p0 .. p0 + 3, p0 = clamp(sx, 0, in_w - 4)), which holds every pixel the
// quad's clamped positions clamp(sx + k, 0, in_w - 1) name -- so the fix-up is a shuffle of the
// lane's own LDS quad (no global load, whose wait would also drain the DMA in flight).  The
// caller brackets it with barriers.
__device__ __forceinline__ void mf_fix_edges(char* buf, int rows, int nq, int xlo, int in_w, int wave, int lane) {
    const int sx = xlo + 4 * lane;
    if (lane >= nq || (sx >= 0 && sx + 4 <= in_w)) return;
    const int p0 = min(max(sx, 0), in_w - 4);
    int idx[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) idx[k] = min(max(sx + k, 0), in_w - 1) - p0;
    for (int r = wave; r < rows; r += 2) {
        uint4* q = reinterpret_cast<uint4*>(buf + ((size_t)r * nq + lane) * 16);
        const uint4 v = *q;
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = idx[k] == 0 ? v.x : idx[k] == 1 ? v.y : idx[k] == 2 ? v.z : v.w;
        *q = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

// The block pipeline of one workgroup.  Blocks alternate between buf0 and buf1; blocks 0 and
// 1 are posted up front and block b + 2 as soon as every wave is done with block b, so two
// blocks' LDS-DMA are in flight at the start and one while each block's products run.  buf0 / buf1 are
// __restrict__: the compiler then sees the ds_reads of one buffer as independent of the DMA
// into the other and waits only for the DMA they depend on (a counted vmcnt, not vmcnt(0)).
template <int NK, int NRB>
__device__ __forceinline__ void mf_main(char* __restrict__ buf0, char* __restrict__ buf1,
                                        const uint8_t* __restrict__ in, int in_pitch, int in_w, int in_h, int xlo,
                                        int ylo, int nr, int nrb, int nq, int lds_cols, uint32_t loff, int kb,
                                        int wave, int lane, const mf_h8* bh, const mf_h8 (*av)[2], mf_f16* Y) {
    const int h = lane >> 5, l32 = lane & 31;
    // quads straddling the right picture edge (xlo is a multiple of 4, so only when in_w is not);
    // columns wholly outside carry weight 0 (build_scale_frags folds the edge taps)
    const bool edge = (in_w & 3) != 0 && xlo + 4 * nq > in_w;  // workgroup-uniform
    // (block 0 landed and block 1 posted by the caller)
    // channel c of pixels (2p, 2p+1) -> f16 pair: byte c of each into the low byte of a half
    constexpr uint32_t kSel[3] = {0x0c040c00u, 0x0c050c01u, 0x0c060c02u};  // B, G, R
#pragma unroll
    for (int b = 0; b < NRB; ++b) {
        if (b > 0 && b >= nrb) break;  // nrb >= 1
        char* cur = (b & 1) ? buf1 : buf0;
        // this wave's DMA of block b retired (__syncthreads() alone does not wait for LDS-DMA).
        // Vector-memory operations retire in order, so waiting until no more than block b + 1's
        // own DMA instructions (if posted) remain leaves exactly those in flight: block 0 starts
        // its products as soon as it and the weight fragments have landed.
        wait_vm_le(b + 1 < nrb ? mf_stage_count(32 * (b + 1), nr, wave) : 0);
        mf_barrier();
        if (b == 0) MF_STAMP(2, __builtin_amdgcn_s_memtime());
        if (b == 1) MF_STAMP(4, __builtin_amdgcn_s_memtime());
        if (edge) {  // quads crossing the left/right image edge: per-pixel clamp
            mf_fix_edges(cur, min(32, nr - 32 * b), nq, xlo, in_w, wave, lane);
            mf_barrier();
        }
        const uint32_t* rp =
            reinterpret_cast<const uint32_t*>(cur) + min(l32, nr - 1 - 32 * b) * lds_cols + kb + 8 * h;
        // the block's K window read once (one LDS latency, not one per step and channel), then
        // the three channels' X chains interleaved step by step, so consecutive MFMAs never wait
        // on each other's accumulator; X -> f16 of one channel overlaps the others' products
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        u32x4 pv[NK][2];
#pragma unroll
        for (int s = 0; s < NK; ++s) {
            pv[s][0] = *reinterpret_cast<const u32x4*>(rp + 16 * s);
            pv[s][1] = *reinterpret_cast<const u32x4*>(rp + 16 * s + 4);
        }
        // all reads in flight before the first product (else the scheduler re-serialises them
        // behind the MFMAs to save registers: one LDS latency per step); whole 128-bit operands,
        // so the loaded quads stay where ds_read_b128 put them
#pragma unroll
        for (int s = 0; s < NK; ++s) asm volatile("" : "+v"(pv[s][0]), "+v"(pv[s][1]));
        uint4 pk[NK][2];
#pragma unroll
        for (int s = 0; s < NK; ++s)
#pragma unroll
            for (int t = 0; t < 2; ++t) pk[s][t] = make_uint4(pv[s][t].x, pv[s][t].y, pv[s][t].z, pv[s][t].w);
        mf_f16 X[3] = {{}, {}, {}};
#pragma unroll
        for (int s = 0; s < NK; ++s)
#pragma unroll
            for (int c = 0; c < 3; ++c)
                X[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(mf_chan(pk[s][0], pk[s][1], kSel[c]), bh[s], X[c], 0, 0, 0);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            mf_h8 x0, x1;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                x0[j] = (_Float16)X[c][j];
                x1[j] = (_Float16)X[c][8 + j];
            }
            Y[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[b][0], x0, Y[c], 0, 0, 0);
            Y[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[b][1], x1, Y[c], 0, 0, 0);
        }
        if (b == 0) MF_STAMP(3, __builtin_amdgcn_s_memtime());
        if (b + 2 < nrb) {  // block b + 2 into this buffer once every wave has read it
            mf_barrier();
            mf_stage(in, in_pitch, in_h, ylo, 32 * (b + 2), nr, nq, loff, cur, wave, lane);
        }
    }
}

__device__ __forceinline__ void mf_epilogue(const mf_f16* Y, int g0, int wave, int v, int lane, uint8_t* __restrict__ yp,
                                            uint8_t* __restrict__ uvp, int out_pitch, int coded_w, int coded_h);

template <int NK, int NRB>
__global__ __launch_bounds__(128) void k_scale_mfma(const uint8_t* __restrict__ in, int in_pitch, int in_w, int in_h,
                                                    ScaleMfma m, uint8_t* __restrict__ yp, uint8_t* __restrict__ uvp,
                                                    int out_pitch, int coded_w, int coded_h, uint64_t* ts) {
    stamp_start(ts);
    MF_STAMP(0, __builtin_amdgcn_s_memrealtime());
    MF_STAMP(1, __builtin_amdgcn_s_memtime());
    // LDS: two 32-row footprint buffers [32][lds_cols] BGRx (see mf_main)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // XCD-aware tile order: dispatch round-robins workgroups over the 8 XCDs (each with its own
    // L2), so the linear id is remapped to give every XCD a contiguous band of tiles -- the
    // footprint overlap between neighbouring tiles then hits in that XCD's L2
    int tx_, ty_;
    {
        const int nwg = gridDim.x * gridDim.y, id = blockIdx.y * gridDim.x + blockIdx.x;
        const int per = nwg >> 3, xcd = id & 7, k = id >> 3;
        const int lin = k >= per ? id : xcd * per + k;  // the last partial round keeps its id
        tx_ = lin % gridDim.x;
        ty_ = lin / gridDim.x;
    }
    const int g0 = 2 * tx_, gw = min(g0 + wave, m.ngx - 1), v = ty_;
    const int xlo = m.gx[2 * g0];
    const int ylo = m.gy[3 * v], nrb = m.gy[3 * v + 1], nr = m.gy[3 * v + 2];
    const int nq = m.lds_cols >> 2;
    const uint32_t loff = (uint32_t)min(max(xlo + 4 * lane, 0), in_w - 4) * 4;
    // Block 0's DMA, then the weight fragments (ordinary loads), one vmcnt(0) for both, then
    // block 1's DMA: block 1 lands while block 0's products run.  (The compiler's own wait for
    // a fragment counts every vector-memory operation issued after it -- the DMA's count is not
    // static -- so fragments loaded with two blocks in flight behind them would hold block 0's
    // products until block 1 had landed too: profiles/r05_scale/NOTES.md.)
    const size_t buf_bytes = (size_t)32 * m.lds_cols * 4;
    // (NRB >= nrb: every fragment load unconditional -- a load under a branch turns the
    // compiler's wait for it into vmcnt(0) -- those past nrb repeat the last block's)
    const int kb = __builtin_amdgcn_readfirstlane(m.gx[2 * gw]) - xlo;  // (zero fragments past the group's K-steps)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the scalars above, before any DMA
    mf_stage(in, in_pitch, in_h, ylo, 0, nr, nq, loff, smem, wave, lane);
    const uint4* fh = reinterpret_cast<const uint4*>(m.fh) + (size_t)gw * kMfKs * 64 + lane;
    const uint4* fv = reinterpret_cast<const uint4*>(m.fv) + (size_t)v * kMfRb * 128 + lane;
    mf_h8 bh[NK], av[NRB][2];
#pragma unroll
    for (int s = 0; s < NK; ++s) bh[s] = __builtin_bit_cast(mf_h8, fh[s * 64]);
#pragma unroll
    for (int b = 0; b < NRB; ++b) {
        const int bb = min(b, nrb - 1);
        av[b][0] = __builtin_bit_cast(mf_h8, fv[bb * 128]);
        av[b][1] = __builtin_bit_cast(mf_h8, fv[bb * 128 + 64]);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    if (nrb > 1) mf_stage(in, in_pitch, in_h, ylo, 32, nr, nq, loff, smem + buf_bytes, wave, lane);
    mf_f16 Y[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) Y[c] = (mf_f16){};
    mf_main<NK, NRB>(smem, smem + buf_bytes, in, in_pitch, in_w, in_h, xlo, ylo, nr, nrb, nq, m.lds_cols, loff, kb, wave,
                lane, bh, av, Y);
    MF_STAMP(5, __builtin_amdgcn_s_memtime());
    mf_epilogue(Y, g0, wave, v, lane, yp, uvp, out_pitch, coded_w, coded_h);
    MF_STAMP(6, __builtin_amdgcn_s_memtime());
    MF_STAMP(7, __builtin_amdgcn_s_memrealtime());
}

// Output of one wave's 32 x 32 block: Y[c][rho] is output column ox, row oy0 + (rho & 3) + 8 *
// (rho >> 2) + 4h; two rows at a time in packed 16-bit lanes (BT.709 sums stay below 2^16), the
// 2x2 chroma with the neighbouring column's lane
__device__ __forceinline__ void mf_epilogue(const mf_f16* Y, int g0, int wave, int v, int lane, uint8_t* __restrict__ yp,
                                            uint8_t* __restrict__ uvp, int out_pitch, int coded_w, int coded_h) {
    // Store-issue bound (every wave of the grid reaches it at once): 16 byte + 8 short stores per
    // wave became 4 + 4 dword stores.  Per pixel, R, G, B are rounded and saturated into the
    // bytes of one dword (v_cvt_pk_u8_f32), luma is one v_dot4_u32_u8 against the BT.709
    // weights and the 2x2 chroma means go through byte dot products too.  Each group of 4
    // consecutive rows is then transposed inside lane quads (DPP broadcasts + v_perm), so lane
    // k of a quad holds row k's four luma bytes and lanes 0 / 2 the two chroma rows' U V U V.
    // Stores go through buffer resources (row in the scalar offset); lanes with nothing to
    // store -- past the coded width or height, odd lanes for chroma -- get an offset past
    // num_records, which the hardware drops, so no store sits under a branch.
    const int h = lane >> 5, l32 = lane & 31, k = lane & 3;
    const int colq = 32 * (g0 + wave) + (l32 & ~3);  // first column of the lane's quad
    const bool qin = colq < coded_w;                 // (coded_w % 4 == 0: quads wholly in or out)
    constexpr uint32_t kLuma = 47u | (157u << 8) | (16u << 16);  // y709's weights (R, G, B bytes)
    constexpr int kOob = 0x7fffffff;
    const uint32_t pitch = (uint32_t)out_pitch;
    const int rows_left = coded_h - 32 * v;  // rows of this tile inside the picture (> 0, even)
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(yp, (short)0, kOob, 0x00020000);
    const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(uvp, (short)0, kOob, 0x00020000);
    const uint32_t sel01 = (uint32_t)k | ((uint32_t)(4 + k) << 8) | 0x0c0c0000u;   // byte k of B0, B1
    const uint32_t sel23 = 0x00000c0cu | ((uint32_t)k << 16) | ((uint32_t)(4 + k) << 24);  // of B2, B3
    const uint32_t csel = (k & 2) ? 0x07060302u : 0x05040100u;  // high / low halves of C0, C2
#pragma unroll
    for (int m = 0; m < 4; ++m) {  // rows 8m + 4h + 0..3 (accumulator rows rho = 4m .. 4m + 3)
        uint32_t Lp = 0, Cw = 0;
#pragma unroll
        for (int r2 = 0; r2 < 2; ++r2) {
            const int rho = 4 * m + 2 * r2;
            uint32_t P[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                uint32_t q = __builtin_amdgcn_cvt_pk_u8_f32(Y[2][rho + t], 0, 0u);  // R
                q = __builtin_amdgcn_cvt_pk_u8_f32(Y[1][rho + t], 1, q);           // G
                P[t] = __builtin_amdgcn_cvt_pk_u8_f32(Y[0][rho + t], 2, q);        // B
            }
            const uint32_t L0 = (__builtin_amdgcn_udot4(P[0], kLuma, 128u, false) >> 8) + 16;
            const uint32_t L1 = (__builtin_amdgcn_udot4(P[1], kLuma, 128u, false) >> 8) + 16;
            Lp |= (L0 | (L1 << 8)) << (16 * r2);
            // 2x2 chroma: this lane's row pair plus the neighbouring column's (lane ^ 1); the
            // rounded means as bytes R, G, B of one dword (each sum <= 1020: B's shifted-in bits
            // land in R's masked-off high byte); u709 / v709 as differences of byte dot products
            uint32_t rb = (P[0] & 0x00ff00ffu) + (P[1] & 0x00ff00ffu);  // R | B << 16
            uint32_t gg = ((P[0] >> 8) & 0xffu) + ((P[1] >> 8) & 0xffu);
            rb += (uint32_t)__builtin_amdgcn_mov_dpp((int)rb, 0xb1, 0xf, 0xf, false);  // quad_perm 1,0,3,2
            gg += (uint32_t)__builtin_amdgcn_mov_dpp((int)gg, 0xb1, 0xf, 0xf, false);
            const uint32_t C = (((rb + 0x00020002u) >> 2) & 0x00ff00ffu) | (((gg + 2u) >> 2) << 8);
            const int U = ((int)(__builtin_amdgcn_udot4(C, 112u << 16, 128u, false) -
                                 __builtin_amdgcn_udot4(C, 26u | (86u << 8), 0u, false)) >> 8) + 128;
            const int V = ((int)(__builtin_amdgcn_udot4(C, 112u, 128u, false) -
                                 __builtin_amdgcn_udot4(C, (102u << 8) | (10u << 16), 0u, false)) >> 8) + 128;
            Cw |= ((uint32_t)U | ((uint32_t)V << 8)) << (16 * r2);
        }
        // luma: lane k of the quad takes byte k (row 8m + 4h + k) of the four lanes' Lp
        const uint32_t B0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)Lp, 0x00, 0xf, 0xf, false);
        const uint32_t B1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)Lp, 0x55, 0xf, 0xf, false);
        const uint32_t B2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)Lp, 0xaa, 0xf, 0xf, false);
        const uint32_t B3 = (uint32_t)__builtin_amdgcn_mov_dpp((int)Lp, 0xff, 0xf, 0xf, false);
        const uint32_t yw = __builtin_amdgcn_perm(B1, B0, sel01) | __builtin_amdgcn_perm(B3, B2, sel23);
        const int yrow = 8 * m + 4 * h + k;
        const int yvo = (qin && yrow < rows_left) ? (int)((uint32_t)(4 * h + k) * pitch + (uint32_t)colq) : kOob;
        __builtin_amdgcn_raw_buffer_store_b32(yw, yr, yvo, (int)((uint32_t)(32 * v + 8 * m) * pitch), 0);
        // chroma rows 4m + 2h (lane 0 of the quad) and 4m + 2h + 1 (lane 2): U V of columns
        // 4q and 4q + 2, from the even lanes' Cw halves
        const uint32_t C0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)Cw, 0x00, 0xf, 0xf, false);
        const uint32_t C2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)Cw, 0xaa, 0xf, 0xf, false);
        const uint32_t cw = __builtin_amdgcn_perm(C2, C0, csel);
        const int crow = 8 * m + 4 * h + 2 * (k >> 1);  // its first luma row
        const int cvo = (qin && !(k & 1) && crow < rows_left)
                            ? (int)((uint32_t)(2 * h + (k >> 1)) * pitch + (uint32_t)colq)
                            : kOob;
        __builtin_amdgcn_raw_buffer_store_b32(cw, cr, cvo, (int)((uint32_t)(16 * v + 4 * m) * pitch), 0);
    }
}


// ---------------------------------------------------------------- MFMA scaler, strip form
// The block loop of k_scale_strip over a ring of three LDS buffers, unrolled by three so every
// access names its buffer through its own __restrict__ parameter: the compiler then sees a ds_read
// of the block being computed as independent of the LDS-DMA into the other two and waits only for
// its own block (a ring slot picked by a run-time index made it wait vmcnt(0) before every LDS
// read, draining the DMA in flight: 72 us for 4K -> 1080p instead of the pipelined time).
__device__ __forceinline__ void strip_main(char* __restrict__ r0, char* __restrict__ r1, char* __restrict__ r2,
                                           const uint4* __restrict__ fvl, const uint8_t* __restrict__ in,
                                           int in_pitch, int in_w, int in_h, int base, int nb, int nq, int lds_cols,
                                           uint32_t loff, int kb, int nks, int xlo, bool edge, int v0, int v1,
                                           const int* ti, const mf_h8* bh, int g0, int wave, int lane,
                                           uint8_t* __restrict__ yp, uint8_t* __restrict__ uvp, int out_pitch,
                                           int coded_w, int coded_h) {
    const int h = lane >> 5, l32 = lane & 31;
    auto tinfo = [&](int v) {
        const int k = v - v0;
        return k == 0 ? ti[0] : k == 1 ? ti[1] : k == 2 ? ti[2] : ti[3];
    };
    mf_stage(in, in_pitch, in_h, base, 0, 32 * nb, nq, loff, r0, wave, lane);
    if (nb > 1) mf_stage(in, in_pitch, in_h, base, 32, 32 * nb, nq, loff, r1, wave, lane);
    constexpr uint32_t kSel[3] = {0x0c040c00u, 0x0c050c01u, 0x0c060c02u};  // B, G, R
    mf_f16 Y0[3], Y1[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) Y0[c] = Y1[c] = (mf_f16){};
    int vt = v0;  // the oldest tile not stored yet (Y0); vt + 1 accumulates in Y1
    // block i computed from `cur`; block i + 2 posted into `nx` (the slot block i - 1 used)
    auto step = [&](char* __restrict__ cur, char* __restrict__ nx, int i) {
        if (i > 0) mf_barrier();  // every wave is done with block i - 1, whose slot is refilled now
        if (i + 2 < nb) mf_stage(in, in_pitch, in_h, base, 32 * (i + 2), 32 * nb, nq, loff, nx, wave, lane);
        // this wave's DMA of block i retired (the blocks posted after it, 16 row loads each, and
        // an epilogue's stores may stay in flight), then every wave's: the barrier
        const int ahead = min(i + 2, nb - 1) - i;
        if (ahead >= 2)
            __builtin_amdgcn_s_waitcnt(0x8F70);  // vmcnt(32)
        else if (ahead == 1)
            __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16)
        else
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        mf_barrier();
        if (edge) {  // quads crossing the left/right image edge: per-pixel clamp
            mf_fix_edges(cur, 32, nq, xlo, in_w, wave, lane);
            mf_barrier();
        }
        // the tiles block i feeds: vt and / or vt + 1 (wave-uniform)
        const int i0 = tinfo(vt), b0 = i0 & 255, n0 = i0 >> 8;
        const bool use0 = i >= b0 && i < b0 + n0;
        bool use1 = false;
        int b1 = 0;
        if (vt + 1 < v1) {
            const int i1 = tinfo(vt + 1);
            b1 = i1 & 255;
            use1 = i >= b1 && i < b1 + (i1 >> 8);
        }
        const uint32_t* rp = reinterpret_cast<const uint32_t*>(cur) + l32 * lds_cols + kb + 8 * h;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            mf_f16 X = {};
#pragma unroll
            for (int s = 0; s < kMfKs; ++s) {
                if (s > 0 && s >= nks) break;
                const uint4 p0 = *reinterpret_cast<const uint4*>(rp + 16 * s);
                const uint4 p1 = *reinterpret_cast<const uint4*>(rp + 16 * s + 4);
                X = __builtin_amdgcn_mfma_f32_32x32x16_f16(mf_chan(p0, p1, kSel[c]), bh[s], X, 0, 0, 0);
            }
            mf_h8 x0, x1;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                x0[j] = (_Float16)X[j];
                x1[j] = (_Float16)X[8 + j];
            }
            if (use0) {
                const uint4* f = fvl + ((size_t)(vt - v0) * kMfRb + (i - b0)) * 128 + lane;
                Y0[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(mf_h8, f[0]), x0, Y0[c], 0, 0, 0);
                Y0[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(mf_h8, f[64]), x1, Y0[c], 0, 0, 0);
            }
            if (use1) {
                const uint4* f = fvl + ((size_t)(vt + 1 - v0) * kMfRb + (i - b1)) * 128 + lane;
                Y1[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(mf_h8, f[0]), x0, Y1[c], 0, 0, 0);
                Y1[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(mf_h8, f[64]), x1, Y1[c], 0, 0, 0);
            }
        }
        // tile vt complete -- and then possibly vt + 1 too, when its last block is this one as well
        // (a short last tile, or an upscale: both tiles' footprints end in block i)
#pragma unroll 1
        for (int k = 0; k < 2 && vt < v1; ++k) {
            const int ik = tinfo(vt);
            if (i != (ik & 255) + (ik >> 8) - 1) break;
            mf_epilogue(Y0, g0, wave, vt, lane, yp, uvp, out_pitch, coded_w, coded_h);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                Y0[c] = Y1[c];
                Y1[c] = (mf_f16){};
            }
            ++vt;
        }
    };
#pragma unroll 1
    for (int i = 0; i < nb; i += 3) {
        step(r0, r2, i);
        if (i + 1 >= nb) break;
        step(r1, r0, i + 1);
        if (i + 2 >= nb) break;
        step(r2, r1, i + 2);
    }
}


// One workgroup (2 waves, 64 output columns) per column strip of up to kStripMaxT consecutive
// 32-row output tiles.  The strip's input rows are staged in 32-row blocks counted from its first
// tap row through an LDS ring of kStripRing blocks: the DMA of the next two blocks is in flight
// while the current one's products run, and a block that two vertically adjacent tiles both read
// is loaded once and its horizontal product (X = In * Wh) computed once, then accumulated into
// both tiles' vertical products (two accumulator sets: the tile being finished and the next).
// The one-tile-per-workgroup form (k_scale_mfma) ran load, products and stores as three
// machine-wide phases, each workgroup's chain unhidden (profiles/r02_scale/NOTES.md).
__global__ __launch_bounds__(128) void k_scale_strip(const uint8_t* __restrict__ in, int in_pitch, int in_w, int in_h,
                                                     ScaleMfma m, uint8_t* __restrict__ yp, uint8_t* __restrict__ uvp,
                                                     int out_pitch, int coded_w, int coded_h, uint64_t* ts) {
    stamp_start(ts);
    // LDS: the ring of 32-row footprint blocks [32][lds_cols] BGRx, then the strip's vertical
    // weight fragments [tile][kMfRb][2][64 lanes]
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int sx, sy;
    {  // XCD-aware order: every XCD a contiguous band of strips (neighbouring footprints share its L2)
        const int nwg = gridDim.x * gridDim.y, id = blockIdx.y * gridDim.x + blockIdx.x;
        const int per = nwg >> 3, xcd = id & 7, k = id >> 3;
        const int lin = k >= per ? id : xcd * per + k;
        sx = lin % gridDim.x;
        sy = lin / gridDim.x;
    }
    const int T = m.strip;
    const int g0 = 2 * sx, gw = min(g0 + wave, m.ngx - 1);
    const int v0 = sy * T, v1 = min(v0 + T, m.ngy), nt = v1 - v0;
    const int base = m.gy2[3 * v0];
    // the tiles' block ranges, held in scalar registers: a global load inside the block loop would
    // wait vmcnt(0) and so drain the ring's DMA in flight
    int ti[kStripMaxT];
#pragma unroll
    for (int k = 0; k < kStripMaxT; ++k) ti[k] = __builtin_amdgcn_readfirstlane(v0 + k < v1 ? m.gy2[3 * (v0 + k) + 1] : 0);
    auto tinfo = [&](int v) {
        const int k = v - v0;
        return k == 0 ? ti[0] : k == 1 ? ti[1] : k == 2 ? ti[2] : ti[3];
    };
    const int lastinfo = tinfo(v1 - 1);
    const int nb = (lastinfo & 255) + (lastinfo >> 8);  // blocks of the strip
    const int xlo = m.gx[2 * g0];
    const int nq = m.lds_cols >> 2;
    const size_t buf_bytes = (size_t)32 * m.lds_cols * 4;
    uint4* fvl = reinterpret_cast<uint4*>(smem + kStripRing * buf_bytes);
    const uint32_t loff = (uint32_t)min(max(xlo + 4 * lane, 0), in_w - 4) * 4;
    // weights (ordinary loads, all waited for before the first block's DMA is issued, so the DMA
    // waits below count blocks only)
    const int nks = m.gx[2 * gw + 1], kb = m.gx[2 * gw] - xlo;
    const uint4* fh = reinterpret_cast<const uint4*>(m.fh) + (size_t)gw * kMfKs * 64 + lane;
    mf_h8 bh[kMfKs];
#pragma unroll
    for (int s = 0; s < kMfKs; ++s) bh[s] = __builtin_bit_cast(mf_h8, s < nks ? fh[s * 64] : make_uint4(0, 0, 0, 0));
    const uint4* fv = reinterpret_cast<const uint4*>(m.fv2) + (size_t)v0 * kMfRb * 128;
    for (int k = tid; k < nt * kMfRb * 128; k += 128) fvl[k] = fv[k];
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __syncthreads();
    // quads straddling the right picture edge (xlo is a multiple of 4, so only when in_w is not);
    // columns wholly outside carry weight 0 (build_scale_frags folds the edge taps)
    const bool edge = (in_w & 3) != 0 && xlo + 4 * nq > in_w;  // workgroup-uniform
    strip_main(smem, smem + buf_bytes, smem + 2 * buf_bytes, fvl, in, in_pitch, in_w, in_h, base, nb, nq, m.lds_cols,
               loff, kb, nks, xlo, edge, v0, v1, ti, bh, g0, wave, lane, yp, uvp, out_pitch, coded_w, coded_h);
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

// Rows per workgroup: at least one thread per 16-pixel quad, and at most ~128 workgroups so the
// device-scope completion counter sees few atomics (one per workgroup, serialised in L2: with one
// row per workgroup at 4K the 2160 atomics cost ~45 us of a 54 us kernel, profiles/r03_hevc).
static int sse_masked_rows(int w, int h) {
    const int nq = (w + 15) >> 4;
    const int rows = nq >= 256 ? 1 : 256 / nq;
    const int min_rows = (h + 127) / 128;
    return rows > min_rows ? rows : min_rows;
}
int sse_masked_blocks(int w, int h) {
    const int rows = sse_masked_rows(w, h);
    return (h + rows - 1) / rows;
}

void launch_sse_masked(const uint8_t* a, const uint8_t* b, int pitch, int w, int h, int mx0, int my0, int mx1,
                       int my1, unsigned long long* part, unsigned int* counter, unsigned long long* host_out,
                       hipStream_t stream) {
    if ((pitch & 15) != 0 || pitch < ((w + 15) & ~15) || (reinterpret_cast<uintptr_t>(a) & 15) ||
        (reinterpret_cast<uintptr_t>(b) & 15))
        throw std::invalid_argument("sse_masked: planes and pitch must be 16-byte aligned, pitch >= width");
    const int rows = sse_masked_rows(w, h);
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
                         int coded_w, int coded_h, hipStream_t stream, uint64_t* ts) {
    dim3 block(64, 4);
    dim3 grid((coded_w / 4 + 63) / 64, (coded_h / 2 + 3) / 4);
    hipLaunchKernelGGL(k_bgrx_to_nv12, grid, block, 0, stream, bgrx, in_pitch, w, h, y, uv, out_pitch, coded_w,
                       coded_h, ts);
}

bool build_scale_frags(int in_w, int in_h, int out_w, int out_h, int coded_w, int coded_h,
                       const std::vector<int>& x0, const std::vector<float>& wx, int tx, const std::vector<int>& y0,
                       const std::vector<float>& wy, int ty, ScaleFragsHost& out) {
    if (in_w < 4 || out_w < 1 || out_h < 1) return false;
    const int ngx = (coded_w + 31) / 32, ngy = (coded_h + 31) / 32;
    auto f16 = [](float w) {  // weights below the f16 normal range are dropped (matrix-core flush)
        const _Float16 hv = (_Float16)(std::fabs(w) < 6.103515625e-05f ? 0.f : w);
        uint16_t bits;
        std::memcpy(&bits, &hv, 2);
        return std::make_pair(bits, (float)hv);
    };
    std::vector<int> gx(2 * (size_t)ngx), gy(3 * (size_t)ngy);
    std::vector<uint16_t> fh((size_t)ngx * kMfKs * 64 * 8, 0), fv((size_t)ngy * kMfRb * 2 * 64 * 8, 0);
    for (int g = 0; g < ngx; ++g) {
        const int kabs = x0[std::min(32 * g, out_w - 1)] & ~3;
        const int kend = x0[std::min(32 * g + 31, out_w - 1)] + tx;
        const int nks = (kend - kabs + 15) / 16;
        if (nks > kMfKs) return false;
        gx[2 * g] = kabs;
        gx[2 * g + 1] = nks;
        // Taps outside the picture read its edge column (clamp), so their weights are folded
        // into that column's: the K window's columns outside [0, in_w) get weight 0 and the
        // kernels need no per-pixel clamp of the staged footprint (which cost the picture's
        // edge workgroups twice the others' time: profiles/r05_scale/NOTES.md)
        std::vector<float> eff(16 * (size_t)kMfKs);
        for (int c = 0; c < 32; ++c) {
            const int cc = std::min(32 * g + c, out_w - 1);
            std::fill(eff.begin(), eff.end(), 0.f);
            for (int k = 0; k < tx; ++k) {
                const int col = std::min(std::max(x0[cc] + k, 0), in_w - 1) - kabs;
                if (col >= 0 && col < 16 * nks) eff[col] += wx[(size_t)cc * tx + k];
            }
            for (int s = 0; s < nks; ++s)
                for (int hh = 0; hh < 2; ++hh)
                    for (int j = 0; j < 8; ++j)
                        fh[(((size_t)g * kMfKs + s) * 64 + 32 * hh + c) * 8 + j] =
                            f16(kMfHScale * eff[16 * s + 8 * hh + j]).first;
        }
    }
    // k_scale_mfma runs a compile-time K-step count (every group's products unrolled without
    // branches); groups with fewer steps have zero fragments beyond theirs, and the footprint is
    // sized for the instantiated count so those steps read inside the staged rows
    int nk = 0;
    for (int g = 0; g < ngx; ++g) nk = std::max(nk, gx[2 * g + 1]);
    nk = scale_mfma_nk(nk);
    int lds_cols = 0, lds_rows = 0, nrb_max = 1;
    for (int g0 = 0; g0 < ngx; g0 += 2)
        for (int w = 0; w < 2; ++w) {
            const int g = std::min(g0 + w, ngx - 1);
            lds_cols = std::max(lds_cols, gx[2 * g] - gx[2 * g0] + 16 * std::max(nk, gx[2 * g + 1]));
        }
    lds_cols = (lds_cols + 3) & ~3;
    if (((lds_cols >> 2) & 1) == 0) lds_cols += 4;  // odd quad pitch: conflict-free row-parallel b128 reads
    for (int v = 0; v < ngy; ++v) {
        const int ylo = y0[std::min(32 * v, out_h - 1)];
        const int nr = y0[std::min(32 * v + 31, out_h - 1)] + ty - ylo;
        const int nrb = (nr + 31) / 32;
        if (nrb > kMfRb) return false;
        nrb_max = std::max(nrb_max, nrb);
        gy[3 * v] = ylo;
        gy[3 * v + 1] = nrb;
        gy[3 * v + 2] = nr;
        lds_rows = std::max(lds_rows, nr);
        for (int l = 0; l < 64; ++l) {
            const int oy = std::min(32 * v + (l & 31), out_h - 1), hh = l >> 5;
            for (int b = 0; b < nrb; ++b)
                for (int t = 0; t < 2; ++t)
                    for (int j = 0; j < 8; ++j) {
                        // element j of lane half hh in k-step t holds accumulator row
                        // 16t + 8(j >> 2) + 4hh + (j & 3) of the 32-row block
                        const int q = 16 * t + 8 * (j >> 2) + 4 * hh + (j & 3);
                        const int tap = ylo + 32 * b + q - y0[oy];
                        if (tap < 0 || tap >= ty) continue;
                        fv[((((size_t)v * kMfRb + b) * 2 + t) * 64 + l) * 8 + j] = f16(kMfVScale * wy[(size_t)oy * ty + tap]).first;
                    }
        }
    }
    if ((size_t)2 * 32 * lds_cols * 4 > 160 * 1024 || lds_cols > 256) return false;  // one row per wave load
    // strip form: tiles v0 .. v0 + T - 1 share one workgroup; blocks of 32 input rows counted from the
    // strip's first tap row; every block may feed at most two tiles (the kernel's two accumulators)
    std::vector<int> gy2(3 * (size_t)ngy, 0);
    std::vector<uint16_t> fv2((size_t)ngy * kMfRb * 2 * 64 * 8, 0);
    int strip = kStripMaxT;
    if (const char* e = std::getenv("MXDESK_SCALER_STRIP"))  // experiments: cap the tiles per strip
        strip = std::max(1, std::min(kStripMaxT, std::atoi(e)));
    for (; strip >= 1; --strip) {
        bool ok = (size_t)kStripRing * 32 * lds_cols * 4 + (size_t)strip * kMfRb * 128 * 16 <= 152 * 1024;
        for (int v = 0; v < ngy && ok; ++v) {
            const int v0 = v - v % strip;
            const int base = y0[std::min(32 * v0, out_h - 1)];
            const int first = y0[std::min(32 * v, out_h - 1)], last = y0[std::min(32 * v + 31, out_h - 1)] + ty - 1;
            const int blo = (first - base) >> 5, nrb = ((last - base) >> 5) - blo + 1;
            if (nrb > kMfRb || blo > 255) ok = false;
            // tile v + 2 of the strip must not reach back into the blocks of tile v
            if (v >= v0 + 2) {
                const int pfirst = y0[std::min(32 * (v - 2), out_h - 1)];
                const int plast = y0[std::min(32 * (v - 2) + 31, out_h - 1)] + ty - 1;
                (void)pfirst;
                if (((plast - base) >> 5) >= blo) ok = false;
            }
            gy2[3 * v] = base;
            gy2[3 * v + 1] = blo | (nrb << 8);
        }
        if (ok) break;
    }
    if (strip >= 1) {
        for (int v = 0; v < ngy; ++v) {
            const int base = gy2[3 * v], blo = gy2[3 * v + 1] & 255, nrb = gy2[3 * v + 1] >> 8;
            for (int l = 0; l < 64; ++l) {
                const int oy = std::min(32 * v + (l & 31), out_h - 1), hh = l >> 5;
                for (int b = 0; b < nrb; ++b)
                    for (int t = 0; t < 2; ++t)
                        for (int j = 0; j < 8; ++j) {
                            const int q = 16 * t + 8 * (j >> 2) + 4 * hh + (j & 3);
                            const int tap = base + 32 * (blo + b) + q - y0[oy];
                            if (tap < 0 || tap >= ty) continue;
                            fv2[((((size_t)v * kMfRb + b) * 2 + t) * 64 + l) * 8 + j] = f16(kMfVScale * wy[(size_t)oy * ty + tap]).first;
                        }
            }
        }
    } else {
        strip = 0;
    }
    auto align = [](size_t x) { return (x + 255) & ~(size_t)255; };
    out.off_gx = 0;
    out.off_gy = align(gx.size() * 4);
    out.off_fh = out.off_gy + align(gy.size() * 4);
    out.off_fv = out.off_fh + align(fh.size() * 2);
    out.off_gy2 = out.off_fv + align(fv.size() * 2);
    out.off_fv2 = out.off_gy2 + align(gy2.size() * 4);
    out.blob.assign(out.off_fv2 + align(fv2.size() * 2), 0);
    std::memcpy(out.blob.data() + out.off_gy2, gy2.data(), gy2.size() * 4);
    std::memcpy(out.blob.data() + out.off_fv2, fv2.data(), fv2.size() * 2);
    out.strip = strip;
    std::memcpy(out.blob.data() + out.off_gx, gx.data(), gx.size() * 4);
    std::memcpy(out.blob.data() + out.off_gy, gy.data(), gy.size() * 4);
    std::memcpy(out.blob.data() + out.off_fh, fh.data(), fh.size() * 2);
    std::memcpy(out.blob.data() + out.off_fv, fv.data(), fv.size() * 2);
    out.lds_cols = lds_cols;
    out.lds_rows = lds_rows;
    out.nk = nk;
    out.nrb_max = nrb_max;
    out.ngx = ngx;
    out.ngy = ngy;
    (void)in_h;
    return true;
}

void upload_scale_frags(const ScaleFragsHost& h, void** dev, ScaleMfma& mf) {
    if (hipMalloc(dev, h.blob.size()) != hipSuccess) throw std::runtime_error("upload_scale_frags: hipMalloc");
    if (hipMemcpy(*dev, h.blob.data(), h.blob.size(), hipMemcpyHostToDevice) != hipSuccess)
        throw std::runtime_error("upload_scale_frags: hipMemcpy");
    const char* b = static_cast<const char*>(*dev);
    mf.gx = reinterpret_cast<const int*>(b + h.off_gx);
    mf.gy = reinterpret_cast<const int*>(b + h.off_gy);
    mf.fh = b + h.off_fh;
    mf.fv = b + h.off_fv;
    mf.lds_cols = h.lds_cols;
    mf.lds_rows = h.lds_rows;
    mf.nk = h.nk;
    mf.nrb_max = h.nrb_max;
    mf.ngx = h.ngx;
    mf.ngy = h.ngy;
    mf.gy2 = reinterpret_cast<const int*>(b + h.off_gy2);
    mf.fv2 = b + h.off_fv2;
    mf.strip = h.strip;
}

void launch_scale_to_nv12(const uint8_t* bgrx, int in_pitch, int in_w, int in_h, const LanczosTables& t, uint8_t* y,
                          uint8_t* uv, int out_pitch, int coded_w, int coded_h, hipStream_t stream, uint64_t* ts) {
    // the strip form runs only on request (MXDESK_SCALER=strip, or the binding's strip=True): with
    // one 2-wave workgroup per CU it leaves half the SIMDs idle and measured 80 us against the tile
    // kernel's 26 us for 4K -> 1080p (profiles/r05_scale/NOTES.md)
    static const bool want_strip = [] {
        const char* e = std::getenv("MXDESK_SCALER");
        return e && std::string(e) == "strip";
    }();
    if (t.mf.gx && t.mf.strip > 0 && (want_strip || t.mf.force_strip) && t.mf.ngx == (coded_w + 31) / 32 && t.mf.ngy == (coded_h + 31) / 32 &&
        in_w >= 4) {
        const size_t lds = (size_t)kStripRing * 32 * t.mf.lds_cols * 4 + (size_t)t.mf.strip * kMfRb * 128 * 16;
        ensure_func_attr(reinterpret_cast<const void*>(&k_scale_strip), hipFuncAttributeMaxDynamicSharedMemorySize,
                         160 * 1024);
        dim3 grid((coded_w + 63) / 64, (t.mf.ngy + t.mf.strip - 1) / t.mf.strip);
        hipLaunchKernelGGL(k_scale_strip, grid, dim3(128), lds, stream, bgrx, in_pitch, in_w, in_h, t.mf, y, uv,
                           out_pitch, coded_w, coded_h, ts);
        return;
    }
    if (t.mf.gx && t.mf.ngx == (coded_w + 31) / 32 && t.mf.ngy == (coded_h + 31) / 32 && in_w >= 4) {
        const size_t lds = (size_t)2 * 32 * t.mf.lds_cols * 4;
        auto go = [&](auto kern) {
            if (lds > 64 * 1024)
                ensure_func_attr(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                 160 * 1024);
            dim3 grid((coded_w + 63) / 64, (coded_h + 31) / 32);
            hipLaunchKernelGGL(kern, grid, dim3(128), lds, stream, bgrx, in_pitch, in_w, in_h, t.mf, y, uv, out_pitch,
                               coded_w, coded_h, ts);
        };
        auto by_nk = [&](auto nrb) {
            constexpr int R = decltype(nrb)::value;
            switch (t.mf.nk) {  // scale_mfma_nk's values
                case 2: go(&k_scale_mfma<2, R>); break;
                case 3: go(&k_scale_mfma<3, R>); break;
                case 4: go(&k_scale_mfma<4, R>); break;
                case 5: go(&k_scale_mfma<5, R>); break;
                case 6: go(&k_scale_mfma<6, R>); break;
                case 8: go(&k_scale_mfma<8, R>); break;
                default: throw std::logic_error("scale_to_nv12: fragment tables without a K-step count");
            }
        };
        if (t.mf.nrb_max <= 3)
            by_nk(std::integral_constant<int, 3>{});
        else
            by_nk(std::integral_constant<int, kMfRb>{});
        return;
    }
    // worst-case footprint of a tile: scale * tile + taps
    const float sx = (float)in_w / t.out_w, sy = (float)in_h / t.out_h;
    // +4 columns for the aligned start, rounded to whole quads (16-byte LDS stores)
    const int max_nc = (((int)ceilf(sx * kTileW) + t.taps_x + 2 + 4) + 3) & ~3;
    const int max_nr = (int)ceilf(sy * kTileH) + t.taps_y + 2;
    const size_t lds = (((size_t)max_nr * max_nc * 4 + 15) & ~(size_t)15) +
                       ((3 * (size_t)max_nr * kTileW + 7) & ~(size_t)7) * 2 +
                       (size_t)(kTileW * t.taps_x + kTileH * t.taps_y) * 4 + (kTileW + kTileH) * 4;
    const int vec = ((in_pitch & 15) == 0 && (reinterpret_cast<uintptr_t>(bgrx) & 15) == 0) ? 1 : 0;
    if (lds > 160 * 1024) throw std::runtime_error("scale_to_nv12: scale factor too large for one LDS tile");
    if (lds > 64 * 1024) {
        ensure_func_attr(reinterpret_cast<const void*>(&k_scale_to_nv12),
                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    }
    dim3 grid((coded_w + kTileW - 1) / kTileW, (coded_h + kTileH - 1) / kTileH);
    hipLaunchKernelGGL(k_scale_to_nv12, grid, dim3(256), lds, stream, bgrx, in_pitch, in_w, in_h, t, y, uv, out_pitch,
                       coded_w, coded_h, max_nc, max_nr, vec, ts);
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
