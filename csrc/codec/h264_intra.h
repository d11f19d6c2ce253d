// H.264 intra prediction (Intra4x4 9 modes, Intra16x16 4 modes, chroma 4 modes), the
// open-loop intra mode decision and Intra4x4 mode prediction -- shared, __host__ __device__, by
// the HIP kernels (h264_kernels.hip) and the CPU encoder (h264_cpu.cpp), so both make identical
// decisions and reconstructions.  The in-loop deblocking filter lives in h264_deblock.h.
//
// Replaces NVENC's intra toolset and loop filter behind `nvh264enc` (reference
// Dockerfile:210, README.md:21).  Formulas follow ITU-T H.264 8.3.1.2, 8.3.3, 8.3.4.
#pragma once
#include "h264_core.h"

namespace mx {
namespace h264 {

// ---------------------------------------------------------------- Intra4x4 (8.3.1.2)
enum I4Mode : int {
    kI4V = 0, kI4H = 1, kI4DC = 2, kI4DDL = 3, kI4DDR = 4, kI4VR = 5, kI4HD = 6, kI4VL = 7, kI4HU = 8
};

// Neighbour samples of a 4x4 block, read in place from the plane they live in (source or
// reconstruction, global memory or an LDS tile): t(0..7) = p[0..7,-1] (p[4..7,-1] replaced by
// p[3,-1] when the top-right block is unavailable but the top is), l(0..3) = p[-1,0..3],
// tl() = p[-1,-1].  Accessors instead of copied arrays: a private array indexed by the
// prediction formulas lands in GPU scratch memory (profiles/r02_m: 172 B/lane).
struct Nb4 {
    const uint8_t* p;  // the block's top-left sample
    int pitch;
    bool top, left, topleft, topright;
    MXHD int t(int k) const { return p[-pitch + ((k < 4 || topright) ? k : 3)]; }
    MXHD int l(int k) const { return p[k * pitch - 1]; }
    MXHD int tl() const { return p[-pitch - 1]; }
};

MXHD bool i4_mode_ok(int mode, const Nb4& n) {
    switch (mode) {
        case kI4V: case kI4DDL: case kI4VL: return n.top;
        case kI4H: case kI4HU: return n.left;
        case kI4DC: return true;
        default: return n.top && n.left && n.topleft;  // DDR, VR, HD
    }
}

// p[x, y] of 8.3.1.2 for x == -1 or y == -1
MXHD int i4_p(const Nb4& n, int x, int y) {
    if (y < 0) return x < 0 ? n.tl() : n.t(x);
    return n.l(y);
}

// Prediction sample (x, y) of mode `mode` (mode must be available).
MXHD int pred4x4_px(int mode, const Nb4& n, int x, int y) {
    switch (mode) {
        case kI4V: return n.t(x);
        case kI4H: return n.l(y);
        case kI4DC: {
            const int st = n.top ? n.t(0) + n.t(1) + n.t(2) + n.t(3) : 0;
            const int sl = n.left ? n.l(0) + n.l(1) + n.l(2) + n.l(3) : 0;
            if (n.top && n.left) return (st + sl + 4) >> 3;
            if (n.left) return (sl + 2) >> 2;
            if (n.top) return (st + 2) >> 2;
            return 128;
        }
        case kI4DDL:
            if (x == 3 && y == 3) return (n.t(6) + 3 * n.t(7) + 2) >> 2;
            return (n.t(x + y) + 2 * n.t(x + y + 1) + n.t(x + y + 2) + 2) >> 2;
        case kI4DDR:
            if (x > y) return (i4_p(n, x - y - 2, -1) + 2 * i4_p(n, x - y - 1, -1) + i4_p(n, x - y, -1) + 2) >> 2;
            if (x < y) return (i4_p(n, -1, y - x - 2) + 2 * i4_p(n, -1, y - x - 1) + i4_p(n, -1, y - x) + 2) >> 2;
            return (n.t(0) + 2 * n.tl() + n.l(0) + 2) >> 2;
        case kI4VR: {
            const int z = 2 * x - y;
            if (z >= 0 && (z & 1) == 0) return (i4_p(n, x - (y >> 1) - 1, -1) + i4_p(n, x - (y >> 1), -1) + 1) >> 1;
            if (z > 0)
                return (i4_p(n, x - (y >> 1) - 2, -1) + 2 * i4_p(n, x - (y >> 1) - 1, -1) + i4_p(n, x - (y >> 1), -1) +
                        2) >> 2;
            if (z == -1) return (n.l(0) + 2 * n.tl() + n.t(0) + 2) >> 2;
            return (i4_p(n, -1, y - 1) + 2 * i4_p(n, -1, y - 2) + i4_p(n, -1, y - 3) + 2) >> 2;
        }
        case kI4HD: {
            const int z = 2 * y - x;
            if (z >= 0 && (z & 1) == 0) return (i4_p(n, -1, y - (x >> 1) - 1) + i4_p(n, -1, y - (x >> 1)) + 1) >> 1;
            if (z > 0)
                return (i4_p(n, -1, y - (x >> 1) - 2) + 2 * i4_p(n, -1, y - (x >> 1) - 1) + i4_p(n, -1, y - (x >> 1)) +
                        2) >> 2;
            if (z == -1) return (n.l(0) + 2 * n.tl() + n.t(0) + 2) >> 2;
            return (i4_p(n, x - 1, -1) + 2 * i4_p(n, x - 2, -1) + i4_p(n, x - 3, -1) + 2) >> 2;
        }
        case kI4VL:
            if ((y & 1) == 0) return (n.t(x + (y >> 1)) + n.t(x + (y >> 1) + 1) + 1) >> 1;
            return (n.t(x + (y >> 1)) + 2 * n.t(x + (y >> 1) + 1) + n.t(x + (y >> 1) + 2) + 2) >> 2;
        default: {  // kI4HU
            const int z = x + 2 * y;
            if (z < 5 && (z & 1) == 0) return (n.l(y + (x >> 1)) + n.l(y + (x >> 1) + 1) + 1) >> 1;
            if (z < 5) return (n.l(y + (x >> 1)) + 2 * n.l(y + (x >> 1) + 1) + n.l(y + (x >> 1) + 2) + 2) >> 2;
            if (z == 5) return (n.l(2) + 3 * n.l(3) + 2) >> 2;
            return n.l(3);
        }
    }
}

// Availability of the top-right 4x4 neighbour of luma block (bx, by) inside a macroblock
// (decoding order, 6.4.11.4): blocks whose top-right lies later in decoding order, or in
// the macroblock to the right, have none; the top row uses the macroblock above-right.
MXHD bool i4_topright_inside(int bx, int by) {
    // true if the top-right block is inside this MB (or above-right MB for by == 0) and
    // already decoded
    if (by == 0) return true;  // depends on the above / above-right MB (checked by caller)
    if (bx == 3) return false;
    // blkIdx order: the top-right of (1,1) is (2,0) = blk 4, after blk 3; likewise (1,3) / (3,*)
    if (bx == 1 && (by == 1 || by == 3)) return false;
    return true;
}

// ---------------------------------------------------------------- Intra16x16 / chroma
// Neighbours of a 16x16 luma block (size 16) or an 8x8 chroma block (size 8) read in place:
// `step` 2 / `comp` select one plane of interleaved NV12 chroma.
struct NbMb {
    const uint8_t* p;  // the block's top-left sample (of component comp)
    int pitch, step;
    bool top, left, topleft;
    MXHD int t(int k) const { return p[-pitch + k * step]; }
    MXHD int l(int k) const { return p[k * pitch - step]; }
    MXHD int tl() const { return p[-pitch - step]; }
};

enum I16Mode : int { kI16V = 0, kI16H = 1, kI16DC = 2, kI16Plane = 3 };
enum ChromaMode : int { kCDC = 0, kCH = 1, kCV = 2, kCPlane = 3 };

MXHD bool i16_mode_ok(int mode, const NbMb& n) {
    if (mode == kI16V) return n.top;
    if (mode == kI16H) return n.left;
    if (mode == kI16DC) return true;
    return n.top && n.left && n.topleft;
}
MXHD bool chroma_mode_ok(int mode, const NbMb& n) {
    if (mode == kCV) return n.top;
    if (mode == kCH) return n.left;
    if (mode == kCDC) return true;
    return n.top && n.left && n.topleft;
}

struct PredMb {  // precomputed DC / plane parameters of one 16x16 (luma) or 8x8 (chroma) block
    int mode;
    int dc[4];     // luma: dc[0]; chroma: per 4x4 block (raster)
    int a, b, c;   // plane
};

MXHD PredMb prep_i16(int mode, const NbMb& n) {
    PredMb p{};
    p.mode = mode;
    if (mode == kI16DC) {
        int st = 0, sl = 0;  // unavailable neighbours are never read (they may lie outside the plane)
        for (int i = 0; i < 16; ++i) {
            st += n.top ? n.t(i) : 0;
            sl += n.left ? n.l(i) : 0;
        }
        p.dc[0] = (n.top && n.left) ? (st + sl + 16) >> 5 : n.left ? (sl + 8) >> 4 : n.top ? (st + 8) >> 4 : 128;
    } else if (mode == kI16Plane) {
        int H = 0, V = 0;
        for (int k = 0; k < 8; ++k) {
            H += (k + 1) * (n.t(8 + k) - (k == 7 ? n.tl() : n.t(6 - k)));
            V += (k + 1) * (n.l(8 + k) - (k == 7 ? n.tl() : n.l(6 - k)));
        }
        p.a = 16 * (n.l(15) + n.t(15));
        p.b = (5 * H + 32) >> 6;
        p.c = (5 * V + 32) >> 6;
    }
    return p;
}
MXHD int pred16_px(const PredMb& p, const NbMb& n, int x, int y) {
    switch (p.mode) {
        case kI16V: return n.t(x);
        case kI16H: return n.l(y);
        case kI16DC: return p.dc[0];
        default: return clip255((p.a + p.b * (x - 7) + p.c * (y - 7) + 16) >> 5);
    }
}

MXHD PredMb prep_chroma(int mode, const NbMb& n) {
    PredMb p{};
    p.mode = mode;
    if (mode == kCDC) {
        for (int blk = 0; blk < 4; ++blk) {
            const int xo = (blk & 1) * 4, yo = (blk >> 1) * 4;
            const int st = n.top ? n.t(xo) + n.t(xo + 1) + n.t(xo + 2) + n.t(xo + 3) : 0;
            const int sl = n.left ? n.l(yo) + n.l(yo + 1) + n.l(yo + 2) + n.l(yo + 3) : 0;
            int v;
            if ((xo == 0 && yo == 0) || (xo > 0 && yo > 0)) {
                v = (n.top && n.left) ? (st + sl + 4) >> 3 : n.left ? (sl + 2) >> 2 : n.top ? (st + 2) >> 2 : 128;
            } else if (xo > 0) {  // yo == 0: top row prefers the top samples
                v = n.top ? (st + 2) >> 2 : n.left ? (sl + 2) >> 2 : 128;
            } else {  // xo == 0, yo > 0: left column prefers the left samples
                v = n.left ? (sl + 2) >> 2 : n.top ? (st + 2) >> 2 : 128;
            }
            p.dc[blk] = v;
        }
    } else if (mode == kCPlane) {
        int H = 0, V = 0;
        for (int k = 0; k < 4; ++k) {
            H += (k + 1) * (n.t(4 + k) - (k == 3 ? n.tl() : n.t(2 - k)));
            V += (k + 1) * (n.l(4 + k) - (k == 3 ? n.tl() : n.l(2 - k)));
        }
        p.a = 16 * (n.l(7) + n.t(7));
        p.b = (34 * H + 32) >> 6;
        p.c = (34 * V + 32) >> 6;
    }
    return p;
}
MXHD int predc_px(const PredMb& p, const NbMb& n, int x, int y) {
    switch (p.mode) {
        case kCDC: {  // select, not a dynamic index (that would put PredMb in GPU scratch)
            const int q = (y >> 2) * 2 + (x >> 2);
            return q == 0 ? p.dc[0] : q == 1 ? p.dc[1] : q == 2 ? p.dc[2] : p.dc[3];
        }
        case kCH: return n.l(y);
        case kCV: return n.t(x);
        default: return clip255((p.a + p.b * (x - 3) + p.c * (y - 3) + 16) >> 5);
    }
}

// ---------------------------------------------------------------- SATD / decision
// Sum of absolute 4x4 Hadamard coefficients of a residual block, halved (SATD).
MXHD uint32_t satd4x4(const int* d) {
    int h[16];
    hadamard4x4(d, h);
    uint32_t s = 0;
    for (int i = 0; i < 16; ++i) s += (uint32_t)(h[i] < 0 ? -h[i] : h[i]);
    return (s + 1) >> 1;
}

constexpr uint32_t kCostInf = 0x3fffffffu;

// Per-macroblock open-loop intra costs (SATD against predictions built from SOURCE
// neighbours, so every macroblock is analysed independently and in parallel):
struct IntraCosts {
    uint32_t c4[16][9];  // [blkIdx][I4 mode], kCostInf when unavailable
    uint32_t c16[4];     // [I16 mode]
    uint32_t cc[4];      // [chroma mode] (Cb + Cr)
};

struct IntraDecision {
    int type;        // kMbI16x16 / kMbI4x4
    int i16_mode;
    int chroma_mode;
    uint8_t i4[16];  // modes, raster (by * 4 + bx)
    uint32_t cost;   // luma + chroma, lambda-weighted
    uint32_t cost_luma;
};

// Estimated predicted-mode flag cost inside the MB: internal neighbours use the modes just
// chosen; neighbours in other macroblocks are unknown during the parallel analysis and are
// taken as DC (the actual coding uses the true predictor).
MXHD IntraDecision decide_intra(const IntraCosts& c, int qp, bool allow4 = true) {
    const uint32_t lam = (uint32_t)lambda_sad(qp);
    IntraDecision d{};
    int m4[16];  // raster
    uint32_t cost4 = 6 * lam;  // I_NxN signalling overhead vs I16x16 (16 mode fields + cbp)
    for (int b = 0; b < 16; ++b) {
        const int bx = kBlkX[b], by = kBlkY[b];
        const int ma = bx > 0 ? m4[by * 4 + bx - 1] : kI4DC;
        const int mb = by > 0 ? m4[(by - 1) * 4 + bx] : kI4DC;
        const int pm = ma < mb ? ma : mb;
        uint32_t best = kCostInf;
        int bm = kI4DC;
        for (int m = 0; m < 9; ++m) {
            if (c.c4[b][m] >= kCostInf) continue;
            const uint32_t v = c.c4[b][m] + lam * (m == pm ? 1u : 4u);
            if (v < best) {
                best = v;
                bm = m;
            }
        }
        m4[by * 4 + bx] = bm;
        cost4 += best;
    }
    uint32_t cost16 = kCostInf;
    int b16 = kI16DC;
    for (int m = 0; m < 4; ++m) {
        if (c.c16[m] >= kCostInf) continue;
        const uint32_t v = c.c16[m] + lam * 2u;
        if (v < cost16) {
            cost16 = v;
            b16 = m;
        }
    }
    uint32_t costc = kCostInf;
    int bc = kCDC;
    for (int m = 0; m < 4; ++m) {
        if (c.cc[m] >= kCostInf) continue;
        const uint32_t v = c.cc[m] + lam * (uint32_t)ue_len((uint32_t)m);
        if (v < costc) {
            costc = v;
            bc = m;
        }
    }
    if (!allow4) cost4 = kCostInf;  // EncoderConfig::intra4x4 = 0: Intra16x16 only (faster IDR reconstruction)
    d.type = cost4 < cost16 ? 2 /* kMbI4x4 */ : 1 /* kMbI16x16 */;
    d.i16_mode = b16;
    d.chroma_mode = bc;
    for (int i = 0; i < 16; ++i) d.i4[i] = (uint8_t)m4[i];
    d.cost_luma = cost4 < cost16 ? cost4 : cost16;
    d.cost = d.cost_luma + costc;
    return d;
}

// predIntra4x4PredMode (8.3.1.1) given the neighbour modes (-1 = "use DC": neighbour MB
// unavailable -> dcPredModePredictedFlag, or not coded in Intra4x4).
MXHD int i4_pred_mode(int mode_a, int mode_b, bool a_avail, bool b_avail) {
    if (!a_avail || !b_avail) return kI4DC;
    const int a = mode_a < 0 ? kI4DC : mode_a, b = mode_b < 0 ? kI4DC : mode_b;
    return a < b ? a : b;
}

// ---------------------------------------------------------------- neighbours from a picture
// Availability of the four neighbour macroblocks (picture + slice bounds), as mb_avail().
// Intra4x4 block (bx, by) availability inside / around the macroblock (6.4.11.4):
MXHD bool i4_left_avail(int bx, bool mb_left) { return bx > 0 || mb_left; }
MXHD bool i4_top_avail(int by, bool mb_top) { return by > 0 || mb_top; }
MXHD bool i4_topleft_avail(int bx, int by, bool mb_left, bool mb_top, bool mb_topleft) {
    if (bx > 0 && by > 0) return true;
    if (bx > 0) return mb_top;
    if (by > 0) return mb_left;
    return mb_topleft;
}
MXHD bool i4_topright_avail(int bx, int by, bool mb_top, bool mb_topright) {
    if (by == 0) return bx < 3 ? mb_top : mb_topright;
    return i4_topright_inside(bx, by);
}

// Neighbour accessor of luma 4x4 block (bx, by) of the macroblock at (x0, y0) of a plane
// (`pl`, pitch) -- the source picture for the open-loop analysis, the reconstruction for coding.
MXHD Nb4 nb4_from_plane(const uint8_t* pl, int pitch, int x0, int y0, int bx, int by, bool mb_left, bool mb_top,
                        bool mb_topright, bool mb_topleft) {
    Nb4 n;
    n.p = pl + (y0 + 4 * by) * pitch + x0 + 4 * bx;
    n.pitch = pitch;
    n.left = i4_left_avail(bx, mb_left);
    n.top = i4_top_avail(by, mb_top);
    n.topleft = i4_topleft_avail(bx, by, mb_left, mb_top, mb_topleft);
    n.topright = n.top && i4_topright_avail(bx, by, mb_top, mb_topright);
    return n;
}

// Neighbours of the whole 16x16 luma block (size 16) or an 8x8 chroma block (size 8, plane of
// interleaved NV12 chroma: step 2, `comp` 0 = Cb / 1 = Cr).
MXHD NbMb nbmb_from_plane(const uint8_t* pl, int pitch, int x0, int y0, int size, int step, int comp, bool mb_left,
                          bool mb_top, bool mb_topleft) {
    (void)size;
    NbMb n;
    n.p = pl + y0 * pitch + x0 * step + comp;
    n.pitch = pitch;
    n.step = step;
    n.left = mb_left;
    n.top = mb_top;
    n.topleft = mb_topleft;
    return n;
}

// ---------------------------------------------------------------- open-loop analysis costs
// SATD of Intra4x4 mode m of block b (blkIdx) predicted from SOURCE neighbours; kCostInf if
// the mode is unavailable.  src points at the macroblock's top-left source sample.
MXHD uint32_t i4_cost(const uint8_t* src, int pitch, int x0, int y0, int b, int m, bool mb_left, bool mb_top,
                      bool mb_topright, bool mb_topleft) {
    const int bx = kBlkX[b], by = kBlkY[b];
    const Nb4 n = nb4_from_plane(src, pitch, x0, y0, bx, by, mb_left, mb_top, mb_topright, mb_topleft);
    if (!i4_mode_ok(m, n)) return kCostInf;
    int d[16];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c)
            d[r * 4 + c] = (int)src[(y0 + 4 * by + r) * pitch + x0 + 4 * bx + c] - pred4x4_px(m, n, c, r);
    return satd4x4(d);
}

// SATD of 4x4 luma block b (raster index rb = by*4+bx) under Intra16x16 mode p.mode.
MXHD uint32_t i16_block_cost(const uint8_t* src, int pitch, int x0, int y0, int rb, const PredMb& p, const NbMb& n) {
    const int bx = rb & 3, by = rb >> 2;
    int d[16];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c)
            d[r * 4 + c] =
                (int)src[(y0 + 4 * by + r) * pitch + x0 + 4 * bx + c] - pred16_px(p, n, 4 * bx + c, 4 * by + r);
    return satd4x4(d);
}

// SATD of chroma 4x4 block cb (raster 2x2) of component comp under chroma mode p.mode.
MXHD uint32_t chroma_block_cost(const uint8_t* suv, int pitch, int xc0, int yc0, int comp, int cb, const PredMb& p,
                                const NbMb& n) {
    const int bx = cb & 1, by = cb >> 1;
    int d[16];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c)
            d[r * 4 + c] = (int)suv[(yc0 + 4 * by + r) * pitch + 2 * (xc0 + 4 * bx + c) + comp] -
                           predc_px(p, n, 4 * bx + c, 4 * by + r);
    return satd4x4(d);
}

// Intra4x4 modes packed two per byte (raster block order).
MXHD int i4_get(const uint8_t* modes, int rb) { return (modes[rb >> 1] >> (4 * (rb & 1))) & 15; }
MXHD void i4_set(uint8_t* modes, int rb, int m) {
    modes[rb >> 1] = (uint8_t)((modes[rb >> 1] & ~(15 << (4 * (rb & 1)))) | (m << (4 * (rb & 1))));
}

// Inverse 4x4 zig-zag: raster position -> scan index.
constexpr uint8_t kZigzagInv4x4[16] = {0, 1, 5, 6, 2, 4, 7, 12, 3, 8, 11, 13, 9, 10, 14, 15};

// Intra is only considered for P macroblocks whose inter prediction is poor (luma SATD above
// 8 per sample): static and well-predicted desktop areas skip the analysis entirely (at 4 per
// sample a fifth of the 1080p desktop's MBs were analysed for no measurable gain: profiles/r02_intra).
constexpr uint32_t kIntraMinInterCost = 256u * 8u;
MXHD bool intra_candidate(uint32_t inter_cost) { return inter_cost > kIntraMinInterCost; }

// Intra vs inter in P pictures: the open-loop intra cost (clean source neighbours) is
// optimistic, so it has to win by 1/8 plus the macroblock-type overhead.
// Gain of switching a P macroblock to intra: the open-loop intra cost (clean source
// neighbours) is optimistic, so it has to win by 1/8 plus the macroblock-type overhead.
// Noise-like content (intra SATD >= 32 per sample: neither prediction works) stays inter, at
// its adaptive-quantisation QP.  0 = stays inter.
MXHD int32_t intra_gain(uint32_t intra_luma_cost, uint32_t inter_cost, int qp) {
    if (intra_luma_cost >= 256u * 32u) return 0;
    const uint32_t pen = intra_luma_cost + (intra_luma_cost >> 3) + 4u * (uint32_t)lambda_sad(qp);
    return inter_cost > pen ? (int32_t)(inter_cost - pen) : 0;
}

// Intra macroblocks of a P picture are made mutually independent: an MB switches only if its
// gain is a strict local maximum among its 8 neighbours (ties to the lower address).  No intra
// MB then has an intra neighbour, so every one predicts from final inter reconstructions and
// all of them are coded in parallel (k_intra_p) -- no reconstruction wavefront in P pictures;
// a region that wants more intra MBs gets the rest in the next picture.  Switched MBs are coded
// at the frame QP.
MXHD bool intra_selected(const int32_t* gain, int mb_w, int mb_h, int mbx, int mby) {
    const int i = mby * mb_w + mbx;
    const int32_t g = gain[i];
    if (g <= 0) return false;
    for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
            const int x = mbx + dx, y = mby + dy;
            if ((dx | dy) == 0 || x < 0 || y < 0 || x >= mb_w || y >= mb_h) continue;
            const int j = y * mb_w + x;
            const int32_t h = gain[j];
            if (h > g || (h == g && j < i)) return false;
        }
    return true;
}

}  // namespace h264
}  // namespace mx
