// VP8 (RFC 6386) encoder core shared, __host__ __device__, by the HIP kernels (vp8_kernels.hip)
// and the CPU oracle encoder (vp8_cpu.cpp): transforms, quantisation, the 16x16 / chroma intra
// predictors with VP8's frame-edge rules, the token / mode / motion-vector trees and their fixed
// probabilities, and (host side) the boolean entropy encoder.
//
// Replaces the reference's `vp8enc` (libvpx) element behind WEBRTC_ENCODER=vp8enc (reference
// README.md:21,35; libvpx-dev at Dockerfile:453).  The bit-exact decode side lives in
// mxdesk/codec/vp8_decoder.py; key frames are additionally decoded by libwebp through Pillow.
//
// Coding subset (what this encoder emits): key frames of 16x16-predicted macroblocks (DC / V / H /
// TM luma, DC / V / H / TM chroma, Y2 second-order block); inter frames of 16x16 inter macroblocks
// predicting from the last frame with quarter-sample vectors (ZEROMV / NEARESTMV / NEARMV / NEWMV);
// inter frames segmented (9.3) by the temporal classes of the H.264 encoder's adaptive
// quantisation -- four segment quantisers, a per-macroblock segment map -- key frames one
// quantiser; the normal loop filter with per-segment levels (section 15; opt-in, on or adaptive:
// on for coherent motion, vp8_encoder.h LfDecision); token partitions by MB row; coefficient
// probabilities updated per frame from the token statistics of frame n - kStatsLag (vp8_encoder.h).
#pragma once
#include <stdint.h>

#include "vp8_tables.h"

#ifndef MXV8
#define MXV8 __host__ __device__ __forceinline__
#endif

namespace mx {
namespace vp8 {

constexpr int kBlocks = 25;        // 16 Y, 4 U, 4 V, Y2
constexpr int kCoefPerMb = 25 * 16;  // int16 levels per macroblock, zigzag (scan) order per block
constexpr int kY2 = 24;

enum YMode : uint8_t { kDcPred = 0, kVPred = 1, kHPred = 2, kTmPred = 3, kInter = 4 };
enum MvMode : uint8_t { kMvZero = 0, kMvNearest = 1, kMvNear = 2, kMvNew = 3 };

// Per-macroblock record written by the analysis (GPU or CPU), read by the bitstream writer.
struct Vp8Mb {
    int16_t mvx, mvy;  // luma vector, 1/8-sample units (even: quarter-sample luma vectors)
    uint8_t ymode;     // YMode
    uint8_t uvmode;    // DC / V / H / TM
    uint8_t seg;       // segment (Seg; 0 in key frames)
    uint8_t pad1;
    uint32_t nz;       // bit b: block b (0..24) has a non-zero level
    uint32_t slot;     // GPU: index of the macroblock's levels in the compacted level buffer
    uint32_t sse[3];   // GPU: Y / U / V distortion over the display area
    uint32_t pad2;
};
static_assert(sizeof(Vp8Mb) == 32, "Vp8Mb layout");

// zigzag scan -> raster position, coefficient bands (13.3)
constexpr uint8_t kZigzag[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
constexpr uint8_t kBand[17] = {0, 1, 2, 3, 6, 4, 5, 6, 6, 6, 6, 6, 6, 6, 6, 7, 0};
// DCT extra-bit probabilities (13.2) for categories 1..6 and their base values
constexpr uint8_t kPcat1[1] = {159};
constexpr uint8_t kPcat2[2] = {165, 145};
constexpr uint8_t kPcat3[3] = {173, 148, 140};
constexpr uint8_t kPcat4[4] = {176, 155, 140, 135};
constexpr uint8_t kPcat5[5] = {180, 157, 141, 134, 130};
constexpr uint8_t kPcat6[11] = {254, 254, 243, 230, 196, 177, 153, 140, 133, 130, 129};
// key-frame mode probabilities (11.2) and inter-frame defaults (16.1)
constexpr uint8_t kKfYModeProb[4] = {145, 156, 163, 128};
constexpr uint8_t kKfUvModeProb[3] = {142, 114, 183};
constexpr uint8_t kYModeProb[4] = {112, 86, 140, 37};
constexpr uint8_t kUvModeProb[3] = {162, 101, 204};
// motion vector entropy (17.2): default contexts and update probabilities
constexpr uint8_t kMvDefault[2][19] = {
    {162, 128, 225, 146, 172, 147, 214, 39, 156, 128, 129, 132, 75, 145, 178, 206, 239, 254, 254},
    {164, 128, 204, 170, 119, 235, 140, 230, 228, 128, 130, 130, 74, 148, 180, 203, 236, 254, 254}};
constexpr uint8_t kMvUpdateProbs[2][19] = {
    {237, 246, 253, 253, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 250, 250, 252, 254, 254},
    {231, 243, 245, 253, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 251, 251, 254, 254, 254}};
// inter mode contexts (16.3): probability of each mv_ref_tree branch by neighbour count
constexpr uint8_t kModeContexts[6][4] = {{7, 1, 1, 143},     {14, 18, 14, 107}, {135, 64, 57, 68},
                                         {60, 56, 128, 65},  {159, 134, 128, 34}, {234, 188, 128, 28}};

MXV8 int v8_clamp255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

// ---------------------------------------------------------------- segments (9.3)
// Inter-frame segments = the temporal classes of h264_mb.h (temporal_class / aq3_mb_qp): the
// segment quantiser is the class's QP offset from the frame QP, sent as absolute quantiser
// indices; segment ids are coded in every inter frame's macroblock headers.
enum Seg : uint8_t { kSegNormal = 0, kSegStatic = 1, kSegPersistent = 2, kSegChanging = 3 };
constexpr int kNumSegs = 4;
// h264_mb.h TClass (kTcNormal 0, kTcPersistent 1, kTcChanging 2, kTcStatic 3) -> Seg, and back
MXV8 int seg_of_tclass(int tc) { return tc == 1 ? kSegPersistent : (tc == 2 ? kSegChanging : (tc == 3 ? kSegStatic : kSegNormal)); }
MXV8 int tclass_of_seg(int seg) { return seg == kSegPersistent ? 1 : (seg == kSegChanging ? 2 : (seg == kSegStatic ? 3 : 0)); }

// ---------------------------------------------------------------- quantisers (14.1, 9.6)
struct Quant {
    int y1dc, y1ac, y2dc, y2ac, uvdc, uvac;
};
MXV8 Quant quant_of(int q) {
    q = q < 0 ? 0 : (q > 127 ? 127 : q);
    Quant r;
    r.y1dc = kDcQ[q];
    r.y1ac = kAcQ[q];
    r.y2dc = 2 * kDcQ[q];
    r.y2ac = kAcQ[q] * 155 / 100;
    if (r.y2ac < 8) r.y2ac = 8;
    r.uvdc = kDcQ[q] > 132 ? 132 : kDcQ[q];
    r.uvac = kAcQ[q];
    return r;
}
// Frame quantiser index for the shared rate controller's QP: the VP8 AC step closest to twice
// the H.264 step (VP8's transform output is 8x the sample scale, H.264's 4x), so the rate model
// of h264::EncoderCommon carries over.
MXV8 int qindex_for_qp(int qp) {
    // 2 * 0.625 * 2^(qp/6) in 1/16 units without floating point: table of 2^(k/6) * 1024
    constexpr int kPow[6] = {1024, 1149, 1290, 1448, 1625, 1825};
    const long long target16 = (long long)20 * kPow[qp % 6] * (1ll << (qp / 6)) / 1024;  // step * 16
    int best = 0;
    long long bd = 1ll << 62;
    for (int q = 0; q < 128; ++q) {
        const long long d = (long long)kAcQ[q] * 16 - target16;
        const long long a = d < 0 ? -d : d;
        if (a < bd) {
            bd = a;
            best = q;
        }
    }
    return best;
}
// Dead-zone quantiser: level = sign * floor(|c| / q + 1/3) (the decoder only sees the levels).
MXV8 int quantize(int c, int q) {
    const int a = c < 0 ? -c : c;
    int l = (3 * a + q) / (3 * q);
    if (l > 2048) l = 2048;  // DCT_MAX_VALUE: the largest category-6 token
    return c < 0 ? -l : l;
}

// ---------------------------------------------------------------- transforms (14.3, 14.4)
// Forward 4x4 DCT (encoder side; any approximation decodes -- this is libvpx's integer form).
MXV8 void fdct4x4(const int* in, int* out) {  // in: residual raster 4x4; out: raster coefficients
    int t[16];
    for (int i = 0; i < 4; ++i) {
        const int* ip = in + 4 * i;
        const int a1 = (ip[0] + ip[3]) * 8, b1 = (ip[1] + ip[2]) * 8;
        const int c1 = (ip[1] - ip[2]) * 8, d1 = (ip[0] - ip[3]) * 8;
        t[4 * i + 0] = a1 + b1;
        t[4 * i + 2] = a1 - b1;
        t[4 * i + 1] = (c1 * 2217 + d1 * 5352 + 14500) >> 12;
        t[4 * i + 3] = (d1 * 2217 - c1 * 5352 + 7500) >> 12;
    }
    for (int i = 0; i < 4; ++i) {
        const int a1 = t[i] + t[12 + i], b1 = t[4 + i] + t[8 + i];
        const int c1 = t[4 + i] - t[8 + i], d1 = t[i] - t[12 + i];
        out[i] = (a1 + b1 + 7) >> 4;
        out[8 + i] = (a1 - b1 + 7) >> 4;
        out[4 + i] = ((c1 * 2217 + d1 * 5352 + 12000) >> 16) + (d1 != 0 ? 1 : 0);
        out[12 + i] = (d1 * 2217 - c1 * 5352 + 51000) >> 16;
    }
}
// Inverse 4x4 DCT (normative, 14.3): coefficients (raster) -> residual (raster).
MXV8 void idct4x4(const int* in, int* out) {
    constexpr int c8 = 20091, s8 = 35468;  // cos(pi/8)*sqrt2 - 1, sin(pi/8)*sqrt2 (Q16)
    int t[16];
    for (int i = 0; i < 4; ++i) {  // columns
        const int i0 = in[i], i4 = in[4 + i], i8 = in[8 + i], i12 = in[12 + i];
        const int a1 = i0 + i8, b1 = i0 - i8;
        const int c1 = ((i4 * s8) >> 16) - (i12 + ((i12 * c8) >> 16));
        const int d1 = (i4 + ((i4 * c8) >> 16)) + ((i12 * s8) >> 16);
        t[i] = a1 + d1;
        t[12 + i] = a1 - d1;
        t[4 + i] = b1 + c1;
        t[8 + i] = b1 - c1;
    }
    for (int i = 0; i < 4; ++i) {  // rows
        const int* ip = t + 4 * i;
        const int a1 = ip[0] + ip[2], b1 = ip[0] - ip[2];
        const int c1 = ((ip[1] * s8) >> 16) - (ip[3] + ((ip[3] * c8) >> 16));
        const int d1 = (ip[1] + ((ip[1] * c8) >> 16)) + ((ip[3] * s8) >> 16);
        out[4 * i + 0] = (a1 + d1 + 4) >> 3;
        out[4 * i + 3] = (a1 - d1 + 4) >> 3;
        out[4 * i + 1] = (b1 + c1 + 4) >> 3;
        out[4 * i + 2] = (b1 - c1 + 4) >> 3;
    }
}
// Forward Walsh-Hadamard of the 16 luma DC values (raster by block) -> Y2 coefficients (raster).
MXV8 void fwht4x4(const int* in, int* out) {
    int t[16];
    for (int i = 0; i < 4; ++i) {
        const int* ip = in + 4 * i;
        const int a1 = (ip[0] + ip[2]) * 4, d1 = (ip[1] + ip[3]) * 4;
        const int c1 = (ip[1] - ip[3]) * 4, b1 = (ip[0] - ip[2]) * 4;
        t[4 * i + 0] = a1 + d1 + (a1 != 0 ? 1 : 0);
        t[4 * i + 1] = b1 + c1;
        t[4 * i + 2] = b1 - c1;
        t[4 * i + 3] = a1 - d1;
    }
    for (int i = 0; i < 4; ++i) {
        const int a1 = t[i] + t[8 + i], d1 = t[4 + i] + t[12 + i];
        const int c1 = t[4 + i] - t[12 + i], b1 = t[i] - t[8 + i];
        int a2 = a1 + d1, b2 = b1 + c1, c2 = b1 - c1, d2 = a1 - d1;
        a2 += a2 < 0;
        b2 += b2 < 0;
        c2 += c2 < 0;
        d2 += d2 < 0;
        out[i] = (a2 + 3) >> 3;
        out[4 + i] = (b2 + 3) >> 3;
        out[8 + i] = (c2 + 3) >> 3;
        out[12 + i] = (d2 + 3) >> 3;
    }
}
// Inverse Walsh-Hadamard (normative, 14.3): Y2 coefficients (raster) -> the 16 blocks' DC values.
MXV8 void iwht4x4(const int* in, int* out) {
    int t[16];
    for (int i = 0; i < 4; ++i) {
        const int a1 = in[i] + in[12 + i], b1 = in[4 + i] + in[8 + i];
        const int c1 = in[4 + i] - in[8 + i], d1 = in[i] - in[12 + i];
        t[i] = a1 + b1;
        t[4 + i] = c1 + d1;
        t[8 + i] = a1 - b1;
        t[12 + i] = d1 - c1;
    }
    for (int i = 0; i < 4; ++i) {
        const int* ip = t + 4 * i;
        const int a1 = ip[0] + ip[3], b1 = ip[1] + ip[2];
        const int c1 = ip[1] - ip[2], d1 = ip[0] - ip[3];
        out[4 * i + 0] = (a1 + b1 + 3) >> 3;
        out[4 * i + 1] = (c1 + d1 + 3) >> 3;
        out[4 * i + 2] = (a1 - b1 + 3) >> 3;
        out[4 * i + 3] = (d1 - c1 + 3) >> 3;
    }
}

// ---------------------------------------------------------------- intra prediction (12.2, 12.3)
// Neighbour samples of an n x n block (n = 16 luma, 8 chroma) with VP8's frame-edge values: the
// row above the picture is 127 (its corner too), the column left of it 129.
struct Edge {
    int above[16];
    int left[16];
    int corner;  // above-left
    bool have_above, have_left;
};
// predicted sample (x, y) of mode m (DC / V / H / TM)
MXV8 int pred_px(int mode, const Edge& e, int n, int x, int y, int dc) {
    switch (mode) {
        case kVPred:
            return e.above[x];
        case kHPred:
            return e.left[y];
        case kTmPred:
            return v8_clamp255(e.left[y] + e.above[x] - e.corner);
        default:
            return dc;
    }
}
// DC value (12.2): the mean of the available edges, 128 when neither is inside the picture.
MXV8 int dc_of(const Edge& e, int n) {
    int s = 0, cnt = 0;
    if (e.have_above) {
        for (int i = 0; i < n; ++i) s += e.above[i];
        ++cnt;
    }
    if (e.have_left) {
        for (int i = 0; i < n; ++i) s += e.left[i];
        ++cnt;
    }
    if (cnt == 0) return 128;
    const int shift = (n == 16 ? 3 : 2) + cnt;  // log2 of the number of summed samples
    return (s + (1 << (shift - 1))) >> shift;
}

// ---------------------------------------------------------------- inter prediction (18.3)
// Six-tap sub-sample filters by 1/8-sample phase; luma vectors are quarter-sample (even phases),
// chroma vectors (luma / 2) reach every phase.
constexpr int kSubpel[8][6] = {{0, 0, 128, 0, 0, 0},     {0, -6, 123, 12, -1, 0}, {2, -11, 108, 36, -8, 1},
                               {0, -9, 93, 50, -6, 0},   {3, -16, 77, 77, -16, 3}, {0, -6, 50, 93, -9, 0},
                               {1, -8, 36, 108, -11, 2}, {0, -1, 12, 123, -6, 0}};
// Predicted sample at integer position (x, y) + phase (fx, fy) / 8: horizontal pass over the six
// rows y-2 .. y+3 (each rounded and clamped to 8 bits), then the vertical pass -- libvpx's 2-D
// filter, exact for phase 0 (the 128 tap).  at(x, y): reference sample with edge extension.
template <class F>
MXV8 int sixtap_px(const F& at, int x, int y, int fx, int fy) {
    int s = 0;
    for (int r = 0; r < 6; ++r) {
        int h = 0;
        for (int k = 0; k < 6; ++k) h += kSubpel[fx][k] * at(x - 2 + k, y - 2 + r);
        s += kSubpel[fy][r] * v8_clamp255((h + 64) >> 7);
    }
    return v8_clamp255((s + 64) >> 7);
}
// Chroma vector (1/8 chroma samples) of a 16x16 luma vector in 1/8 luma samples (18.4):
// halved, rounded away from zero.
MXV8 int chroma_mv(int v) { return (v + (v < 0 ? -1 : 1)) / 2; }

// ---------------------------------------------------------------- loop filter (15)
// The normal filter (filter_type 0, sharpness 0, no mode / reference level deltas): per
// macroblock a level from its segment; macroblock edges take the wide filter (15.3 MB edges),
// the inner 4x4 edges (only in macroblocks with a non-zero coefficient -- all 16x16-predicted
// here) the subblock filter.  Arithmetic as libvpx's C reference (the RFC's normative source):
// the edge test 2|p0-q0| + |p1-q1|/2 <= limit, interior |p_i - p_i+1| <= interior limit, high
// edge variance |p1-p0| or |q1-q0| above the frame-type threshold.
struct LfParams {
    int mblim, blim, lim, hev;  // MB-edge / subblock-edge limits, interior limit, hev threshold
};
MXV8 LfParams lf_params(int level, bool key) {
    LfParams f;
    f.lim = level < 1 ? 1 : level;  // interior limit (sharpness 0)
    f.mblim = (level + 2) * 2 + f.lim;
    f.blim = level * 2 + f.lim;
    f.hev = key ? (level >= 40 ? 2 : (level >= 15 ? 1 : 0)) : (level >= 40 ? 3 : (level >= 20 ? 2 : (level >= 15 ? 1 : 0)));
    return f;
}
MXV8 int lf_s8(int v) { return v < -128 ? -128 : (v > 127 ? 127 : v); }
MXV8 int lf_abs(int v) { return v < 0 ? -v : v; }
// p[0..7] = p3 p2 p1 p0 q0 q1 q2 q3 across the edge
MXV8 bool lf_mask(const int* p, int lim, int elim) {
    return lf_abs(p[3] - p[4]) * 2 + (lf_abs(p[2] - p[5]) >> 1) <= elim && lf_abs(p[0] - p[1]) <= lim &&
           lf_abs(p[1] - p[2]) <= lim && lf_abs(p[2] - p[3]) <= lim && lf_abs(p[7] - p[6]) <= lim &&
           lf_abs(p[6] - p[5]) <= lim && lf_abs(p[5] - p[4]) <= lim;
}
// macroblock edge: p2 .. q2 change (without high edge variance; else p0 / q0 as the subblock filter)
MXV8 void lf_mb_edge(int* p, const LfParams& f) {
    if (!lf_mask(p, f.lim, f.mblim)) return;
    const int ps2 = p[1] - 128, ps1 = p[2] - 128, ps0 = p[3] - 128, qs0 = p[4] - 128, qs1 = p[5] - 128, qs2 = p[6] - 128;
    const bool hev = lf_abs(p[2] - p[3]) > f.hev || lf_abs(p[5] - p[4]) > f.hev;
    const int w = lf_s8(lf_s8(ps1 - qs1) + 3 * (qs0 - ps0));
    if (hev) {
        p[4] = lf_s8(qs0 - (lf_s8(w + 4) >> 3)) + 128;
        p[3] = lf_s8(ps0 + (lf_s8(w + 3) >> 3)) + 128;
        return;
    }
    int a = lf_s8((27 * w + 63) >> 7);
    p[4] = lf_s8(qs0 - a) + 128;
    p[3] = lf_s8(ps0 + a) + 128;
    a = lf_s8((18 * w + 63) >> 7);
    p[5] = lf_s8(qs1 - a) + 128;
    p[2] = lf_s8(ps1 + a) + 128;
    a = lf_s8((9 * w + 63) >> 7);
    p[6] = lf_s8(qs2 - a) + 128;
    p[1] = lf_s8(ps2 + a) + 128;
}
// subblock edge: p1 .. q1 change (p0 / q0 only with high edge variance)
MXV8 void lf_sub_edge(int* p, const LfParams& f) {
    if (!lf_mask(p, f.lim, f.blim)) return;
    const int ps1 = p[2] - 128, ps0 = p[3] - 128, qs0 = p[4] - 128, qs1 = p[5] - 128;
    const bool hev = lf_abs(p[2] - p[3]) > f.hev || lf_abs(p[5] - p[4]) > f.hev;
    const int a = lf_s8((hev ? lf_s8(ps1 - qs1) : 0) + 3 * (qs0 - ps0));
    const int f1 = lf_s8(a + 4) >> 3, f2 = lf_s8(a + 3) >> 3;
    p[4] = lf_s8(qs0 - f1) + 128;
    p[3] = lf_s8(ps0 + f2) + 128;
    if (!hev) {
        const int o = (f1 + 1) >> 1;
        p[5] = lf_s8(qs1 - o) + 128;
        p[2] = lf_s8(ps1 + o) + 128;
    }
}
// Level of a segment coded at quantiser index q (libvpx's encoder searches it per frame; a fixed
// map here): num / 16 of the index, at most 63.
MXV8 int lf_level_for(int q, int num) {
    const int l = (q * num) >> 4;
    return l > 63 ? 63 : (l < 0 ? 0 : l);
}
constexpr int kLfNumDefault = 5;

// One plane of one macroblock (n x n samples at (x0, y0); `step` 1 for luma, 2 for a component of
// interleaved chroma): left edge, inner vertical edges, top edge, inner horizontal edges (15.1).
inline void lf_plane_mb(uint8_t* base, int step, int pitch, int x0, int y0, int n, bool left, bool top, bool inner,
                        const LfParams& f) {
    auto at = [&](int x, int y) -> uint8_t& { return base[(size_t)y * pitch + (size_t)x * step]; };
    int p[8];
    auto vedge = [&](int xe, bool mb) {
        for (int r = 0; r < n; ++r) {
            for (int k = 0; k < 8; ++k) p[k] = at(xe - 4 + k, y0 + r);
            if (mb)
                lf_mb_edge(p, f);
            else
                lf_sub_edge(p, f);
            for (int k = 1; k < 7; ++k) at(xe - 4 + k, y0 + r) = (uint8_t)p[k];
        }
    };
    auto hedge = [&](int ye, bool mb) {
        for (int c = 0; c < n; ++c) {
            for (int k = 0; k < 8; ++k) p[k] = at(x0 + c, ye - 4 + k);
            if (mb)
                lf_mb_edge(p, f);
            else
                lf_sub_edge(p, f);
            for (int k = 1; k < 7; ++k) at(x0 + c, ye - 4 + k) = (uint8_t)p[k];
        }
    };
    if (left) vedge(x0, true);
    if (inner)
        for (int e = 4; e < n; e += 4) vedge(x0 + e, false);
    if (top) hedge(y0, true);
    if (inner)
        for (int e = 4; e < n; e += 4) hedge(y0 + e, false);
}
// The whole reconstructed frame in place, macroblocks in raster order (the serial reference of
// k_vp8_lf): level levels[segment] (0: the macroblock is not filtered), inner edges where the
// macroblock has a non-zero coefficient.  y / uv (interleaved chroma) `pitch` wide.
inline void loop_filter_frame(uint8_t* y, uint8_t* uv, int pitch, int mb_w, int mb_h, const Vp8Mb* mbs,
                              const int* levels, bool key) {
    for (int mby = 0; mby < mb_h; ++mby)
        for (int mbx = 0; mbx < mb_w; ++mbx) {
            const Vp8Mb& m = mbs[mby * mb_w + mbx];
            const int level = levels[m.seg & 3];
            if (!level) continue;
            const LfParams f = lf_params(level, key);
            const bool inner = m.nz != 0;
            lf_plane_mb(y, 1, pitch, mbx * 16, mby * 16, 16, mbx > 0, mby > 0, inner, f);
            for (int c = 0; c < 2; ++c) lf_plane_mb(uv + c, 2, pitch, mbx * 8, mby * 8, 8, mbx > 0, mby > 0, inner, f);
        }
}

// ---------------------------------------------------------------- macroblock coding (shared)
// Quantise + reconstruct the 16 luma blocks of a macroblock with a second-order Y2 block.
// res: residual 16x16 raster; pred: prediction 16x16 raster; lv: output levels [25][16] in scan
// order (blocks 0..15 and 24 written); rec: output samples 16x16 raster; returns the nz bits.
MXV8 uint32_t code_luma16(const int* res, const int* pred, const Quant& Q, int16_t* lv, int* rec) {
    int dc[16], coef[16][16];
    for (int b = 0; b < 16; ++b) {
        const int bx = b & 3, by = b >> 2;
        int in[16];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) in[i * 4 + j] = res[(by * 4 + i) * 16 + bx * 4 + j];
        fdct4x4(in, coef[b]);
        dc[b] = coef[b][0];
    }
    int y2[16], y2q[16], y2d[16], dcr[16];
    fwht4x4(dc, y2);
    uint32_t nz = 0;
    for (int k = 0; k < 16; ++k) {
        const int pos = kZigzag[k];
        const int l = quantize(y2[pos], k == 0 ? Q.y2dc : Q.y2ac);
        lv[kY2 * 16 + k] = (int16_t)l;
        y2q[pos] = l * (k == 0 ? Q.y2dc : Q.y2ac);
        if (l) nz |= 1u << kY2;
    }
    (void)y2d;
    iwht4x4(y2q, dcr);
    for (int b = 0; b < 16; ++b) {
        int dq[16];
        lv[b * 16] = 0;
        dq[0] = dcr[b];
        for (int k = 1; k < 16; ++k) {
            const int pos = kZigzag[k];
            const int l = quantize(coef[b][pos], Q.y1ac);
            lv[b * 16 + k] = (int16_t)l;
            dq[pos] = l * Q.y1ac;
            if (l) nz |= 1u << b;
        }
        int r[16];
        idct4x4(dq, r);
        const int bx = b & 3, by = b >> 2;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                const int o = (by * 4 + i) * 16 + bx * 4 + j;
                rec[o] = v8_clamp255(pred[o] + r[i * 4 + j]);
            }
    }
    return nz;
}
// One chroma component (8x8): blocks 16..19 (U) or 20..23 (V).
MXV8 uint32_t code_chroma8(const int* res, const int* pred, const Quant& Q, int16_t* lv, int* rec, int first_block) {
    uint32_t nz = 0;
    for (int b = 0; b < 4; ++b) {
        const int bx = b & 1, by = b >> 1;
        int in[16], coef[16], dq[16], r[16];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) in[i * 4 + j] = res[(by * 4 + i) * 8 + bx * 4 + j];
        fdct4x4(in, coef);
        for (int k = 0; k < 16; ++k) {
            const int pos = kZigzag[k];
            const int q = k == 0 ? Q.uvdc : Q.uvac;
            const int l = quantize(coef[pos], q);
            lv[(first_block + b) * 16 + k] = (int16_t)l;
            dq[pos] = l * q;
            if (l) nz |= 1u << (first_block + b);
        }
        idct4x4(dq, r);
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                const int o = (by * 4 + i) * 8 + bx * 4 + j;
                rec[o] = v8_clamp255(pred[o] + r[i * 4 + j]);
            }
    }
    return nz;
}

}  // namespace vp8
}  // namespace mx
