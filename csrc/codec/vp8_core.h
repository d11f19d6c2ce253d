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
// TM luma, DC / V / H / TM chroma, Y2 second-order block) and B_PRED macroblocks (ten 4x4
// sub-block modes under the key-frame contexts kKfBModeProb, each sub-block predicted from the
// ones reconstructed before it, no Y2 block), chosen per macroblock by prediction SAD plus
// lambda * mode bits; inter frames of 16x16 inter macroblocks
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

enum YMode : uint8_t { kDcPred = 0, kVPred = 1, kHPred = 2, kTmPred = 3, kInter = 4, kBPred = 5 };
// B_PRED sub-block modes in the bmode tree's leaf order (= the index order of kKfBModeProb):
// B_DC "0", B_TM "10", B_VE "110", B_HE "11100", B_RD "111010", B_VR "111011", B_LD "111101",
// B_VL "1111100", B_HD "11111010", B_HU "11111011"
enum BMode : uint8_t { kBDc = 0, kBTm, kBVe, kBHe, kBRd, kBVr, kBLd, kBVl, kBHd, kBHu, kNumBModes };
enum MvMode : uint8_t { kMvZero = 0, kMvNearest = 1, kMvNear = 2, kMvNew = 3 };

// Per-macroblock record written by the analysis (GPU or CPU), read by the bitstream writer.
struct Vp8Mb {
    int16_t mvx, mvy;  // luma vector, 1/8-sample units (even: quarter-sample luma vectors); a key-frame
                       // B_PRED macroblock (no vector) keeps sub-block modes 0..7 here (bmode_of)
    uint8_t ymode;     // YMode
    uint8_t uvmode;    // DC / V / H / TM
    uint8_t seg;       // segment (Seg; 0 in key frames)
    uint8_t pad1;
    uint32_t nz;       // bit b: block b (0..24) has a non-zero level
    uint32_t slot;     // GPU: index of the macroblock's levels in the compacted level buffer
    uint32_t sse[3];   // GPU: Y / U / V distortion over the display area
    uint32_t bmodes_hi;  // B_PRED: sub-block modes 8..15 (4 bits each); inter macroblocks: the luma
                         // prediction SAD (the intra pass's comparison, vp8_intra_candidate)
};
static_assert(sizeof(Vp8Mb) == 32, "Vp8Mb layout");
// B_PRED sub-block modes, 4 bits each in raster order: 0..7 in the vector fields, 8..15 in bmodes_hi
MXV8 int bmode_of(const Vp8Mb& m, int b) {
    const uint32_t w = b < 8 ? ((uint32_t)(uint16_t)m.mvx | ((uint32_t)(uint16_t)m.mvy << 16)) : m.bmodes_hi;
    return (int)((w >> (4 * (b & 7))) & 15u);
}
MXV8 void set_bmodes(Vp8Mb& m, uint32_t lo, uint32_t hi) {
    m.mvx = (int16_t)(uint16_t)(lo & 0xffffu);
    m.mvy = (int16_t)(uint16_t)(lo >> 16);
    m.bmodes_hi = hi;
}
// the sub-block mode a 16x16-predicted macroblock stands for as a B_PRED context (11.3)
MXV8 int implied_bmode(int ymode) {
    return ymode == kVPred ? kBVe : (ymode == kHPred ? kBHe : (ymode == kTmPred ? kBTm : kBDc));
}

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
// -256 log2(p / 256): the cost in 1/256 bit of coding a branch of probability p / 256 (the
// writer's bit_cost256, as a table both encoders share)
constexpr uint16_t kProbCost256[256] = {2048, 2048, 1792, 1642, 1536, 1454, 1386, 1329, 1280, 1236, 1198, 1162, 1130, 1101, 1073, 1048, 1024, 1002, 980, 961, 942, 924, 906, 890, 874, 859, 845, 831, 817, 804, 792, 780, 768, 757, 746, 735, 724, 714, 705, 695, 686, 676, 668, 659, 650, 642, 634, 626, 618, 611, 603, 596, 589, 582, 575, 568, 561, 555, 548, 542, 536, 530, 524, 518, 512, 506, 501, 495, 490, 484, 479, 474, 468, 463, 458, 453, 449, 444, 439, 434, 430, 425, 420, 416, 412, 407, 403, 399, 394, 390, 386, 382, 378, 374, 370, 366, 362, 358, 355, 351, 347, 343, 340, 336, 333, 329, 326, 322, 319, 315, 312, 309, 305, 302, 299, 296, 292, 289, 286, 283, 280, 277, 274, 271, 268, 265, 262, 259, 256, 253, 250, 247, 245, 242, 239, 236, 234, 231, 228, 226, 223, 220, 218, 215, 212, 210, 207, 205, 202, 200, 197, 195, 193, 190, 188, 185, 183, 181, 178, 176, 174, 171, 169, 167, 164, 162, 160, 158, 156, 153, 151, 149, 147, 145, 143, 140, 138, 136, 134, 132, 130, 128, 126, 124, 122, 120, 118, 116, 114, 112, 110, 108, 106, 104, 102, 101, 99, 97, 95, 93, 91, 89, 87, 86, 84, 82, 80, 78, 77, 75, 73, 71, 70, 68, 66, 64, 63, 61, 59, 58, 56, 54, 53, 51, 49, 48, 46, 44, 43, 41, 40, 38, 36, 35, 33, 32, 30, 28, 27, 25, 24, 22, 21, 19, 18, 16, 15, 13, 12, 10, 9, 7, 6, 4, 3, 1};
MXV8 int branch_cost(int prob, int bit) { return (int)kProbCost256[bit ? 256 - prob : prob]; }

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

// ---------------------------------------------------------------- B_PRED sub-blocks (12.3)
// Neighbours of a 4x4 luma sub-block: A[0..7] the row above (4..7 above-right), L[0..3] the column
// to the left, P the corner, with VP8's rules: frame edges 127 above / 129 left (the corner 127 in
// the top row, else 129 in the left column); a macroblock's above-right comes from the row above
// the macroblock -- the above-right macroblock's bottom row, at the right frame edge the above
// macroblock's last sample repeated -- and the right column's lower sub-blocks reuse that same
// above-right (the decoder has not reconstructed anything to their right yet).
struct SubEdge {
    int A[8], L[4], P;
};
MXV8 int avg2(int a, int b) { return (a + b + 1) >> 1; }
MXV8 int avg3(int a, int b, int c) { return (a + 2 * b + c + 2) >> 2; }
// The eight directional modes as 2- / 3-tap averages over one edge array X[15] = L3 L3 L2 L1 L0 P
// A0 .. A7 A7 (bpred_edge): entry s | 16 is avg3(X[s], X[s+1], X[s+2]), s alone avg2(X[s], X[s+1]),
// per mode (B_VE .. B_HU) and sample (y * 4 + x) -- the formulas of RFC 6386 12.3 (subblock_intra_predict),
// tabulated (tools: the table is written out from them; the duplicated L3 / A7 ends give the
// clamped taps of B_HE / B_HU / B_LD)
constexpr uint8_t kBPredTap[8][16] = {
    {21, 22, 23, 24, 21, 22, 23, 24, 21, 22, 23, 24, 21, 22, 23, 24},
    {19, 19, 19, 19, 18, 18, 18, 18, 17, 17, 17, 17, 16, 16, 16, 16},
    {20, 21, 22, 23, 19, 20, 21, 22, 18, 19, 20, 21, 17, 18, 19, 20},
    {5, 6, 7, 8, 20, 21, 22, 23, 19, 5, 6, 7, 18, 20, 21, 22},
    {22, 23, 24, 25, 23, 24, 25, 26, 24, 25, 26, 27, 25, 26, 27, 28},
    {6, 7, 8, 9, 22, 23, 24, 25, 7, 8, 9, 26, 23, 24, 25, 27},
    {4, 20, 21, 22, 3, 19, 4, 20, 2, 18, 3, 19, 1, 17, 2, 18},
    {3, 18, 2, 17, 2, 17, 1, 16, 1, 16, 0, 0, 0, 0, 0, 0}};
MXV8 void bpred_edge(const SubEdge& e, int* X) {
    X[0] = X[1] = e.L[3];
    X[2] = e.L[2];
    X[3] = e.L[1];
    X[4] = e.L[0];
    X[5] = e.P;
    for (int i = 0; i < 8; ++i) X[6 + i] = e.A[i];
    X[14] = e.A[7];
}
// predicted sample (x, y) of mode m from the edge array X (bpred_edge)
MXV8 int bpred_px(int m, const int* X, int x, int y) {
    if (m == kBDc) return (X[6] + X[7] + X[8] + X[9] + X[1] + X[2] + X[3] + X[4] + 4) >> 3;
    if (m == kBTm) return v8_clamp255(X[4 - y] + X[6 + x] - X[5]);
    const int t = kBPredTap[m - 2][y * 4 + x], s = t & 15;
    return (t & 16) ? (X[s] + 2 * X[s + 1] + X[s + 2] + 2) >> 2 : (X[s] + X[s + 1] + 1) >> 1;
}
// Modes this encoder considers for sub-block column bx of macroblock (mbx, mby): in the right column
// not B_VE / B_LD / B_VL (the modes that read the above-right samples) while those come from the
// above-right macroblock -- the GPU's row below then never waits for that macroblock (k_vp8_key).
MXV8 bool bmode_allowed(int m, int bx, int mbx, int mby, int mb_w) {
    return !(bx == 3 && mby > 0 && mbx + 1 < mb_w && (m == kBVe || m == kBLd || m == kBVl));
}
// Cost in 1/256 bit of sub-block mode m through the bmode tree under probabilities p[9]
MXV8 int bmode_tree_cost256(int m, const uint8_t* p) {
    if (m == kBDc) return branch_cost(p[0], 0);
    int c = branch_cost(p[0], 1);
    if (m == kBTm) return c + branch_cost(p[1], 0);
    c += branch_cost(p[1], 1);
    if (m == kBVe) return c + branch_cost(p[2], 0);
    c += branch_cost(p[2], 1);
    if (m == kBHe || m == kBRd || m == kBVr) {
        c += branch_cost(p[3], 0);
        if (m == kBHe) return c + branch_cost(p[4], 0);
        return c + branch_cost(p[4], 1) + branch_cost(p[5], m == kBVr);
    }
    c += branch_cost(p[3], 1);
    if (m == kBLd) return c + branch_cost(p[6], 0);
    c += branch_cost(p[6], 1);
    if (m == kBVl) return c + branch_cost(p[7], 0);
    return c + branch_cost(p[7], 1) + branch_cost(p[8], m == kBHu);
}
// ... after above / left modes a / l in a key frame (kKfBModeProb[a][l]: what the writer codes)
MXV8 int bmode_cost256(int m, int a, int l) { return bmode_tree_cost256(m, kKfBModeProb + (a * kNumBModes + l) * 9); }
// ... without contexts: the plan's estimate (the context-free sub-block mode probabilities VP8 uses
// in inter frames; the plan runs before any neighbour's modes are known)
constexpr uint8_t kBModeProbPlan[9] = {120, 90, 79, 133, 87, 85, 80, 111, 151};
MXV8 int bmode_plan_cost256(int m) { return bmode_tree_cost256(m, kBModeProbPlan); }

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
// the inner 4x4 edges (in macroblocks with a non-zero coefficient, and always in B_PRED
// macroblocks) the subblock filter.  Arithmetic as libvpx's C reference (the RFC's normative source):
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
            const bool inner = m.nz != 0 || m.ymode == kBPred;  // B_PRED: inner edges always (15.1)
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
// One B_PRED luma sub-block b (4x4, no second-order block: type 3, the DC quantised with y1dc):
// res / pred raster 4x4, levels in scan order to lv[b * 16 ..], reconstruction to rec (4x4 raster);
// returns whether a level is non-zero.
MXV8 bool code_sub4(const int* res, const int* pred, const Quant& Q, int16_t* lv, int* rec) {
    int coef[16], dq[16], r[16];
    fdct4x4(res, coef);
    bool nz = false;
    for (int k = 0; k < 16; ++k) {
        const int pos = kZigzag[k];
        const int q = k == 0 ? Q.y1dc : Q.y1ac;
        const int l = quantize(coef[pos], q);
        lv[k] = (int16_t)l;
        dq[pos] = l * q;
        nz |= l != 0;
    }
    idct4x4(dq, r);
    for (int i = 0; i < 16; ++i) rec[i] = v8_clamp255(pred[i] + r[i]);
    return nz;
}
// Sub-block neighbours (SubEdge) of sub-block (bx, by) of macroblock (mbx, mby): `at(x, y)` reads
// the frame's reconstruction at luma (x, y) (this macroblock's earlier sub-blocks included).
template <class F>
MXV8 SubEdge sub_edge(const F& at, int mbx, int mby, int mb_w, int bx, int by) {
    SubEdge e;
    const int x0 = mbx * 16 + bx * 4, y0 = mby * 16 + by * 4;
    const bool top = mby == 0 && by == 0, left = mbx == 0 && bx == 0;
    for (int i = 0; i < 4; ++i) e.A[i] = top ? 127 : at(x0 + i, y0 - 1);
    for (int i = 0; i < 4; ++i) e.L[i] = left ? 129 : at(x0 - 1, y0 + i);
    e.P = top ? 127 : (left ? 129 : at(x0 - 1, y0 - 1));
    // above-right: in the sub-block row above inside the macroblock, else from the row above the
    // macroblock (the right column's lower sub-blocks reuse the macroblock's above-right)
    if (bx < 3 && by > 0) {
        for (int i = 0; i < 4; ++i) e.A[4 + i] = at(x0 + 4 + i, y0 - 1);
    } else if (mby == 0) {
        for (int i = 0; i < 4; ++i) e.A[4 + i] = 127;
    } else if (bx < 3) {
        for (int i = 0; i < 4; ++i) e.A[4 + i] = at(x0 + 4 + i, mby * 16 - 1);
    } else if (mbx + 1 < mb_w) {
        for (int i = 0; i < 4; ++i) e.A[4 + i] = at(mbx * 16 + 16 + i, mby * 16 - 1);
    } else {
        for (int i = 0; i < 4; ++i) e.A[4 + i] = at(mbx * 16 + 15, mby * 16 - 1);
    }
    return e;
}
// Cost in 1/256 bit of a key-frame luma mode (kKfYModeProb tree: B_PRED "0", DC "100", V "101",
// H "110", TM "111")
MXV8 int kf_ymode_cost256(int ymode) {
    const uint8_t* p = kKfYModeProb;
    if (ymode == kBPred) return branch_cost(p[0], 0);
    return branch_cost(p[0], 1) + branch_cost(p[1], ymode >= kHPred) +
           branch_cost(ymode >= kHPred ? p[3] : p[2], ymode == kVPred || ymode == kTmPred);
}

// B_PRED contexts (11.3): the sub-block mode above / left of a macroblock's edge sub-block column
// bx / row by; a 16x16-predicted neighbour stands for its implied mode, outside the frame B_DC.
MXV8 int bctx_above(const Vp8Mb* mbs, int mb_w, int mbx, int mby, int bx) {
    if (mby == 0) return kBDc;
    const Vp8Mb& n = mbs[(mby - 1) * mb_w + mbx];
    return n.ymode == kBPred ? bmode_of(n, 12 + bx) : implied_bmode(n.ymode);
}
MXV8 int bctx_left(const Vp8Mb* mbs, int mb_w, int mbx, int mby, int by) {
    if (mbx == 0) return kBDc;
    const Vp8Mb& n = mbs[mby * mb_w + mbx - 1];
    return n.ymode == kBPred ? bmode_of(n, 4 * by + 3) : implied_bmode(n.ymode);
}
// B_PRED plan of a key-frame macroblock, open loop -- every macroblock at once (k_vp8_bpred_plan:
// one wave per macroblock, ahead of the k_vp8_key wavefront): predictions from the *source*
// neighbours with the frame-edge rules; each sub-block takes the allowed mode (bmode_allowed) of
// least 256 SAD + lam * bmode_plan_cost256 (the lower mode on ties), and the macroblock goes B_PRED
// when their sum plus the B_PRED mode bits is below the best 16x16 mode's 256 SAD + lam * mode bits.
// src(x, y): the source luma.  Modes packed 4 bits each into lo (0..7) / hi (8..15).
template <class S>
MXV8 bool bpred_plan(const S& src, int mbx, int mby, int mb_w, int lam, uint32_t* lo, uint32_t* hi) {
    const int x0 = mbx * 16, y0 = mby * 16;
    Edge e;
    e.have_above = y0 > 0;
    e.have_left = x0 > 0;
    for (int i = 0; i < 16; ++i) {
        e.above[i] = y0 > 0 ? src(x0 + i, y0 - 1) : 127;
        e.left[i] = x0 > 0 ? src(x0 - 1, y0 + i) : 129;
    }
    e.corner = y0 == 0 ? 127 : (x0 == 0 ? 129 : src(x0 - 1, y0 - 1));
    const int dc = dc_of(e, 16);
    uint32_t cost16 = ~0u;
    for (int m = 0; m < 4; ++m) {
        uint32_t sad = 0;
        for (int y = 0; y < 16; ++y)
            for (int x = 0; x < 16; ++x) {
                const int d = src(x0 + x, y0 + y) - pred_px(m, e, 16, x, y, dc);
                sad += (uint32_t)(d < 0 ? -d : d);
            }
        const uint32_t c = 256u * sad + (uint32_t)(lam * kf_ymode_cost256(m));
        if (c < cost16) cost16 = c;
    }
    uint32_t costb = (uint32_t)(lam * kf_ymode_cost256(kBPred));
    *lo = *hi = 0;
    for (int b = 0; b < 16; ++b) {
        const int bx = b & 3, by = b >> 2;
        const SubEdge se = sub_edge(src, mbx, mby, mb_w, bx, by);
        int X[15];
        bpred_edge(se, X);
        uint32_t best = ~0u;
        int bm = kBDc;
        for (int m = 0; m < kNumBModes; ++m) {
            if (!bmode_allowed(m, bx, mbx, mby, mb_w)) continue;
            uint32_t sad = 0;
            for (int y = 0; y < 4; ++y)
                for (int x = 0; x < 4; ++x) {
                    const int d = src(x0 + bx * 4 + x, y0 + by * 4 + y) - bpred_px(m, X, x, y);
                    sad += (uint32_t)(d < 0 ? -d : d);
                }
            const uint32_t c = 256u * sad + (uint32_t)(lam * bmode_plan_cost256(m));
            if (c < best) {
                best = c;
                bm = m;
            }
        }
        costb += best;
        if (b < 8)
            *lo |= (uint32_t)bm << (4 * b);
        else
            *hi |= (uint32_t)bm << (4 * (b - 8));
    }
    return costb < cost16;
}
// B_PRED luma of a planned macroblock, closed loop: the sub-blocks in raster order, each predicted
// in its planned mode from the reconstruction (this macroblock's earlier sub-blocks included) and
// coded (code_sub4) into rec (16x16 raster) and lv blocks 0..15.  src: the macroblock's source
// (pitch); at(x, y): the frame's reconstruction outside the macroblock.  Returns the blocks'
// non-zero bits.
template <class F>
inline uint32_t bpred_code(const uint8_t* src, int pitch, const F& at, int mbx, int mby, int mb_w, const Quant& Q,
                           uint32_t lo, uint32_t hi, int16_t* lv, int* rec) {
    const int x0 = mbx * 16, y0 = mby * 16;
    auto px = [&](int x, int y) {
        return x >= x0 && x < x0 + 16 && y >= y0 && y < y0 + 16 ? rec[(y - y0) * 16 + x - x0] : at(x, y);
    };
    uint32_t nz = 0;
    for (int b = 0; b < 16; ++b) {
        const int bx = b & 3, by = b >> 2;
        const int bm = (int)(((b < 8 ? lo >> (4 * b) : hi >> (4 * (b - 8)))) & 15u);
        int X[15];
        bpred_edge(sub_edge(px, mbx, mby, mb_w, bx, by), X);
        int res[16], pred[16], r4[16];
        for (int y = 0; y < 4; ++y)
            for (int x = 0; x < 4; ++x) {
                pred[y * 4 + x] = bpred_px(bm, X, x, y);
                res[y * 4 + x] = (int)src[(by * 4 + y) * pitch + bx * 4 + x] - pred[y * 4 + x];
            }
        if (code_sub4(res, pred, Q, lv + b * 16, r4)) nz |= 1u << b;
        for (int y = 0; y < 4; ++y)
            for (int x = 0; x < 4; ++x) rec[(by * 4 + y) * 16 + bx * 4 + x] = r4[y * 4 + x];
    }
    return nz;
}

// ---------------------------------------------------------------- intra macroblocks in inter frames
// Two passes after every macroblock was coded inter (its prediction SAD kept in bmodes_hi): a
// macroblock is an intra candidate when its best 16x16 intra mode, predicted from the inter
// reconstruction of its neighbours, beats the inter prediction by more than the mode bits
// (kIntraBits256, lambda-weighted); a candidate switches to intra when none of its causal
// neighbours (left, above, above-left) is a candidate -- then the neighbours it predicts from stay
// inter (their reconstruction is final) and no macroblock that predicts from it switches, so both
// passes run over all macroblocks in parallel (k_vp8_intra_cand / k_vp8_intra_code) and the
// serial encoder reproduces them exactly.
constexpr uint32_t kIntraMinSad = 512;   // inter prediction SAD at or below: never a candidate
constexpr int kIntraBits256 = 8 * 256;    // is_inter_mb + y / uv modes, less the vector, in 1/256 bit
MXV8 bool vp8_intra_candidate(uint32_t inter_sad, uint32_t intra_sad, int lam) {
    return inter_sad > kIntraMinSad && 256ull * intra_sad + (unsigned long long)lam * kIntraBits256 < 256ull * inter_sad;
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
