// HEVC (ISO/IEC 23008-2, Main profile) building blocks shared by the HIP encoder kernels
// (hevc_kernels.hip) and the CPU encoder (hevc_cpu.cpp): CABAC engine and context
// tables, residual / CU syntax, the integer core transform, (de)quantisation, intra
// prediction (all 35 modes) and the 8-tap / 4-tap inter interpolation.  Every function is
// __host__ __device__, so the GPU kernels and the CPU oracle share one definition of
// every bit and every sample.
//
// Coding subset (fixed by the SPS/PPS that hevc_cpu.cpp writes):
//   CTB 32x32 with a coding quadtree (split_cu_flag): a CTB is one CU32 or four CU16.  The
//   encoder analyses 16x16 *units* (kCtb below is the unit size, not the CTB's); a CU32 joins the
//   four units of a CTB when their prediction (type, vector) and QP agree, and its transform tree
//   -- split by size at depth 0 (32 > the 16-sample maximum TB) -- has exactly the units' 16x16
//   trees as its depth-1 nodes, so the units keep their own levels (see "coding tree" below).
//   PU 2Nx2N, TU 16x16 luma / 8x8 chroma; with EncoderConfig.tu_split an inter unit may split its
//   transform tree once more (four 8x8 luma TUs, eight 4x4 chroma TUs), chosen per unit by SSE +
//   lambda * estimated bits; I slices of intra CUs, P slices of skip / merge / AMVP CUs with one
//   reference picture, MaxNumMergeCand 5 (A1 B1 B0 A0 B2), no TMVP, no sign hiding, cu_qp_delta
//   per 16x16 quantization group (adaptive quantisation; QP prediction from the left / above QG
//   inside the CTB, 8.6.1); in-loop deblocking (8.7.2) and sample adaptive offset (8.7.3, band /
//   edge per CTB) on by default.
// Slices and CABAC substreams (CTB aligned): I pictures in slices of up to kMaxSliceRows / 2 CTB
//   rows (the intra wavefront's workgroup); P pictures (default, EncoderConfig.hevc_wpp 0) in up to
//   the level's slice limit of raster runs of CTBs balanced on an estimate of their bin tokens
//   (cu_cost, plan_num_slices), one substream each.  hevc_wpp 1: wavefront parallel processing --
//   slices of hevc_wpp_rows CTB rows, every CTB row a CABAC substream entropy coded by its own GPU
//   wave, starting from the contexts the row above had after its second CTB, with entry points in
//   the slice header.
//
// Replaces NVENC HEVC behind the reference's GStreamer stack (nvh264enc default encoder,
// reference Dockerfile:210 / README.md:21; BASELINE.json config "4K60 HEVC").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef MXHD
#define MXHD __host__ __device__ __forceinline__
#endif

namespace mx {
namespace hevc {

constexpr int kCtb = 16;  // analysis unit (16x16; a CU16, or a quadrant of a CU32)
constexpr int kCtbLog2 = 5;     // CTB 32x32
constexpr int kMinCbLog2 = 4;   // smallest CU 16x16
constexpr int kMaxTbLog2 = 4;   // largest TU 16x16 (a CU32's tree splits at depth 0 by size)
constexpr int kMaxMergeCand = 5;  // MaxNumMergeCand (slice header five_minus_max_num_merge_cand 0)
constexpr int kCoefPerCu = 384;  // 256 luma + 64 Cb + 64 Cr, each TU in scan order

// ---------------------------------------------------------------- scans (6.5.3)
// 4x4 up-right diagonal scan: position n -> (x, y); also used for the 4x4 sub-block
// grid of a 16x16 TU.  kDiag4Inv maps raster (y*4+x) -> n.
constexpr uint8_t kDiag4X[16] = {0, 0, 1, 0, 1, 2, 0, 1, 2, 3, 1, 2, 3, 2, 3, 3};
constexpr uint8_t kDiag4Y[16] = {0, 1, 0, 2, 1, 0, 3, 2, 1, 0, 3, 2, 1, 3, 2, 3};
constexpr uint8_t kDiag4Inv[16] = {0, 2, 5, 9, 1, 4, 8, 12, 3, 7, 11, 14, 6, 10, 13, 15};
// 2x2 diagonal scan (sub-block grid of an 8x8 TU)
constexpr uint8_t kDiag2X[4] = {0, 0, 1, 1};
constexpr uint8_t kDiag2Y[4] = {0, 1, 0, 1};
constexpr uint8_t kDiag2Inv[4] = {0, 2, 1, 3};

// scan index (sub-block * 16 + position) of raster coordinate (x, y) in an NxN TU
// nibble-packed copies (ALU lookups for the wave-uniform CABAC kernel)
constexpr uint64_t kDiag4XP = 0x3323213210210100ull;  // kDiag4X[n] = nibble n
constexpr uint64_t kDiag4YP = 0x3231230123012010ull;
MXHD int diag4x(int n) { return (int)((kDiag4XP >> (4 * n)) & 15); }
MXHD int diag4y(int n) { return (int)((kDiag4YP >> (4 * n)) & 15); }

MXHD int scan_index(int log2n, int x, int y) {
    const int sb = log2n == 4 ? kDiag4Inv[(y >> 2) * 4 + (x >> 2)] : (log2n == 3 ? kDiag2Inv[(y >> 2) * 2 + (x >> 2)] : 0);
    return sb * 16 + kDiag4Inv[(y & 3) * 4 + (x & 3)];
}
MXHD void scan_pos(int log2n, int idx, int* x, int* y) {
    const int sb = idx >> 4, n = idx & 15;
    const int sx = log2n == 4 ? diag4x(sb) : (log2n == 3 ? (sb >> 1) : 0);
    const int sy = log2n == 4 ? diag4y(sb) : (log2n == 3 ? (sb & 1) : 0);
    *x = sx * 4 + diag4x(n);
    *y = sy * 4 + diag4y(n);
}

// scanIdx (7.4.9.11): 0 up-right diagonal, 1 horizontal, 2 vertical.  Intra 4x4 / 8x8 luma TUs and
// 4x4 chroma TUs scan by their prediction mode (intra_scan_idx); every other TU diagonally.  The
// horizontal scan is raster order (sub-blocks of an 8x8 TU too), the vertical one its transpose; the
// 2x2 sub-block grid's diagonal order equals the vertical one.  Levels are stored per TU in the
// TU's own scan order.
MXHD int intra_scan_idx(int mode) { return (mode >= 6 && mode <= 14) ? 2 : ((mode >= 22 && mode <= 30) ? 1 : 0); }
// position (x, y) in a 4x4 sub-block of scan position n
MXHD void sb_pos(int scan, int n, int* x, int* y) {
    if (scan == 0) {
        *x = diag4x(n);
        *y = diag4y(n);
    } else if (scan == 1) {
        *x = n & 3;
        *y = n >> 2;
    } else {
        *x = n >> 2;
        *y = n & 3;
    }
}
// sub-block (x, y) of sub-block scan index i in a TU of log2n (sub-block grid 1x1, 2x2 or 4x4;
// scanIdx 1 / 2 only occur up to 8x8)
MXHD void sb_grid_pos(int log2n, int scan, int i, int* x, int* y) {
    if (log2n == 4) {
        *x = diag4x(i);
        *y = diag4y(i);
    } else if (log2n == 3) {
        *x = scan == 1 ? (i & 1) : (i >> 1);
        *y = scan == 1 ? (i >> 1) : (i & 1);
    } else {
        *x = *y = 0;
    }
}
MXHD void scan_pos_s(int log2n, int scan, int idx, int* x, int* y) {
    int sx, sy, px, py;
    sb_grid_pos(log2n, scan, idx >> 4, &sx, &sy);
    sb_pos(scan, idx & 15, &px, &py);
    *x = sx * 4 + px;
    *y = sy * 4 + py;
}
MXHD int scan_index_s(int log2n, int scan, int x, int y) {
    if (scan == 0) return scan_index(log2n, x, y);
    const int px = x & 3, py = y & 3, sx = x >> 2, sy = y >> 2;
    const int n = scan == 1 ? py * 4 + px : px * 4 + py;
    const int sb = log2n == 3 ? (scan == 1 ? sy * 2 + sx : sx * 2 + sy) : 0;
    return sb * 16 + n;
}

// ---------------------------------------------------------------- core transform (8.6.4.2)
// 32-point matrix coefficients by angle index m (cos(pi*m/64) scaled); every N-point
// matrix row k is row k*32/N of the 32-point matrix.
constexpr uint8_t kCos32[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
                                61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9,  4,  0};
MXHD int dct_coef32(int k, int n) {
    if (k == 0) return 64;
    int m = (k * (2 * n + 1)) & 127;
    if (m > 64) m = 128 - m;
    return m > 32 ? -(int)kCos32[64 - m] : (int)kCos32[m];
}
// N-point matrix entry (row = frequency k, column = sample n)
MXHD int dct_coef(int log2n, int k, int n) { return dct_coef32(k << (5 - log2n), n); }

// Forward 2-D transform (encoder side; HM-style shifts: log2N+bitDepth-9, then log2N+6).
// res: raster NxN residual, out: raster NxN coefficients [v][u].
MXHD void fwd_transform(int log2n, const int* res, int* out) {
    const int N = 1 << log2n;
    const int s1 = log2n - 1, s2 = log2n + 6;  // bitDepth 8
    int tmp[16 * 16];
    for (int y = 0; y < N; ++y)
        for (int k = 0; k < N; ++k) {
            int s = 0;
            for (int n = 0; n < N; ++n) s += dct_coef(log2n, k, n) * res[y * N + n];
            tmp[y * N + k] = (s + (1 << (s1 - 1))) >> s1;
        }
    for (int k2 = 0; k2 < N; ++k2)
        for (int k = 0; k < N; ++k) {
            int s = 0;
            for (int y = 0; y < N; ++y) s += dct_coef(log2n, k2, y) * tmp[y * N + k];
            out[k2 * N + k] = (s + (1 << (s2 - 1))) >> s2;
        }
}

MXHD int clip16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }

// Inverse 2-D transform (normative): columns, clip to 16 bit after (e + 64) >> 7, rows,
// (g + 2048) >> 12.  d: raster coefficients [v][u], r: raster residual.
MXHD void inv_transform(int log2n, const int* d, int* r) {
    const int N = 1 << log2n;
    int g[16 * 16];
    for (int x = 0; x < N; ++x)
        for (int y = 0; y < N; ++y) {
            int s = 0;
            for (int k = 0; k < N; ++k) s += dct_coef(log2n, k, y) * d[k * N + x];
            g[y * N + x] = clip16((s + 64) >> 7);
        }
    for (int y = 0; y < N; ++y)
        for (int x = 0; x < N; ++x) {
            int s = 0;
            for (int k = 0; k < N; ++k) s += dct_coef(log2n, k, x) * g[y * N + k];
            r[y * N + x] = (s + 2048) >> 12;
        }
}

// ---------------------------------------------------------------- quantisation (8.6.2/8.6.3)
constexpr uint16_t kQuantScale[6] = {26214, 23302, 20560, 18396, 16384, 14564};
constexpr uint8_t kLevelScale[6] = {40, 45, 51, 57, 64, 72};

MXHD int quant_coef(int c, int qp, int log2n, bool intra) {
    const int qbits = 14 + qp / 6 + (15 - 8 - log2n);
    const int64_t add = (int64_t)(intra ? 171 : 85) << (qbits - 9);
    const int a = c < 0 ? -c : c;
    int l = (int)(((int64_t)a * kQuantScale[qp % 6] + add) >> qbits);
    l = l > 32767 ? 32767 : l;
    return c < 0 ? -l : l;
}
MXHD int dequant_coef(int level, int qp, int log2n) {
    const int bd = log2n + 3;  // BitDepth + log2(nTbS) - 5
    const int64_t v = (int64_t)level * 16 * kLevelScale[qp % 6] * ((int64_t)1 << (qp / 6)) + (1 << (bd - 1));
    const int64_t s = v >> bd;
    return s < -32768 ? -32768 : (s > 32767 ? 32767 : (int)s);
}
// Table 8-10 (ChromaArrayType 1)
MXHD int chroma_qp(int qp_y, int offset) {
    int q = qp_y + offset;
    q = q < 0 ? 0 : (q > 57 ? 57 : q);
    constexpr uint8_t tab[14] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37};
    if (q < 30) return q;
    if (q > 43) return q - 6;
    return tab[q - 30];
}
MXHD int clip255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

// ---------------------------------------------------------------- intra prediction (8.4.4.2)
// Reference samples: left[k] = p[-1][k-1], top[k] = p[k-1][-1] for k = 0..2N (index 0 is the
// shared corner p[-1][-1]).
constexpr int8_t kIntraAngle[35] = {0,  0,   32,  26,  21,  17,  13,  9,  5,  2,  0,  -2,
                                    -5, -9,  -13, -17, -21, -26, -32, -26, -21, -17, -13, -9,
                                    -5, -2,  0,   2,   5,   9,   13,  17,  21,  26,  32};
MXHD int inv_angle(int angle) {
    // 8192 / angle rounded, for the negative angles of modes 11..25
    switch (angle) {
        case -2: return -4096;
        case -5: return -1638;
        case -9: return -910;
        case -13: return -630;
        case -17: return -482;
        case -21: return -390;
        case -26: return -315;
        default: return -256;  // -32
    }
}

// Substitution process (8.4.4.2.2) for the availability pattern of a block whose left
// column (N samples) may be present and whose corner / top / top-right / below-left are
// absent or present as whole units.  lpx: left column (N), bpx: below-left (N), tpx: top
// (N), trx: top-right (N), corner: p[-1][-1].
MXHD void intra_refs(int N, bool a_left, bool a_bl, bool a_top, bool a_tr, bool a_corner, const uint8_t* lpx,
                     const uint8_t* bpx, const uint8_t* tpx, const uint8_t* trx, int corner, int* left, int* top) {
    // The spec's search order p[-1][2N-1] .. p[-1][-1], p[0][-1] .. p[2N-1][-1] is the linear
    // index i = 0 .. 4N; i < 2N lives in left[2N - i], i == 2N is the corner, i > 2N in top[i - 2N].
    const int n2 = 2 * N, total = 4 * N + 1;
    auto avail = [&](int i) { return i < N ? a_bl : (i < n2 ? a_left : (i == n2 ? a_corner : (i <= 3 * N ? a_top : a_tr))); };
    auto ref = [&](int i) -> int& { return i < n2 ? left[n2 - i] : (i == n2 ? left[0] : top[i - n2]); };
    for (int k = 0; k < N; ++k) {
        left[1 + k] = a_left ? lpx[k] : 0;
        left[1 + N + k] = a_bl ? bpx[k] : 0;
        top[1 + k] = a_top ? tpx[k] : 0;
        top[1 + N + k] = a_tr ? trx[k] : 0;
    }
    left[0] = a_corner ? corner : 0;
    if (!(a_left || a_bl || a_top || a_tr || a_corner)) {
        for (int i = 0; i < total; ++i) ref(i) = 128;
    } else {
        if (!avail(0)) {
            for (int i = 1; i < total; ++i)
                if (avail(i)) {
                    ref(0) = ref(i);
                    break;
                }
        }
        for (int i = 1; i < total; ++i)
            if (!avail(i)) ref(i) = ref(i - 1);
    }
    top[0] = left[0];
}

// Prediction of an NxN block (N = 4..32, 8-bit).  cidx 0 = luma (reference filtering,
// DC / angular edge filters apply), 1/2 = chroma.  pred: raster NxN.
MXHD void intra_predict(int mode, int log2n, int cidx, const int* left_in, const int* top_in, int* pred) {
    const int N = 1 << log2n;
    int left[65], top[65];
    for (int k = 0; k <= 2 * N; ++k) {
        left[k] = left_in[k];
        top[k] = top_in[k];
    }
    // 8.4.4.2.3 filtering (luma only for 4:2:0; strong smoothing disabled)
    if (cidx == 0 && mode != 1 && N != 4) {
        const int d1 = mode > 26 ? mode - 26 : 26 - mode, d2 = mode > 10 ? mode - 10 : 10 - mode;
        const int mind = d1 < d2 ? d1 : d2;
        const int thres = N == 8 ? 7 : (N == 16 ? 1 : 0);
        if (mind > thres) {
            int fl[65], ft[65];
            fl[0] = ft[0] = (left[1] + 2 * left[0] + top[1] + 2) >> 2;
            for (int k = 1; k < 2 * N; ++k) {
                fl[k] = (left[k + 1] + 2 * left[k] + left[k - 1] + 2) >> 2;
                ft[k] = (top[k + 1] + 2 * top[k] + top[k - 1] + 2) >> 2;
            }
            fl[2 * N] = left[2 * N];
            ft[2 * N] = top[2 * N];
            for (int k = 0; k <= 2 * N; ++k) {
                left[k] = fl[k];
                top[k] = ft[k];
            }
        }
    }
    if (mode == 0) {  // planar
        for (int y = 0; y < N; ++y)
            for (int x = 0; x < N; ++x)
                pred[y * N + x] = ((N - 1 - x) * left[1 + y] + (x + 1) * top[1 + N] + (N - 1 - y) * top[1 + x] +
                                   (y + 1) * left[1 + N] + N) >>
                                  (log2n + 1);
        return;
    }
    if (mode == 1) {  // DC
        int s = N;
        for (int k = 1; k <= N; ++k) s += left[k] + top[k];
        const int dc = s >> (log2n + 1);
        for (int i = 0; i < N * N; ++i) pred[i] = dc;
        if (cidx == 0 && N < 32) {
            pred[0] = (left[1] + 2 * dc + top[1] + 2) >> 2;
            for (int x = 1; x < N; ++x) pred[x] = (top[1 + x] + 3 * dc + 2) >> 2;
            for (int y = 1; y < N; ++y) pred[y * N] = (left[1 + y] + 3 * dc + 2) >> 2;
        }
        return;
    }
    const int angle = kIntraAngle[mode];
    int refbuf[3 * 32 + 1];
    int* ref = refbuf + N;  // ref[-N .. 2N]
    const bool vert = mode >= 18;
    const int* mainr = vert ? top : left;  // p along the main direction, index k = ref[k]
    const int* side = vert ? left : top;
    for (int x = 0; x <= N; ++x) ref[x] = mainr[x];
    if (angle < 0) {
        const int lo = (N * angle) >> 5;
        if (lo < -1) {
            const int ia = inv_angle(angle);
            for (int x = lo; x <= -1; ++x) ref[x] = side[(x * ia + 128) >> 8];
        }
    } else {
        for (int x = N + 1; x <= 2 * N; ++x) ref[x] = mainr[x];
    }
    for (int y = 0; y < N; ++y)
        for (int x = 0; x < N; ++x) {
            const int a = vert ? y : x, b = vert ? x : y;  // a: distance along prediction, b: across
            const int idx = ((a + 1) * angle) >> 5, fact = ((a + 1) * angle) & 31;
            const int v = fact ? ((32 - fact) * ref[b + idx + 1] + fact * ref[b + idx + 2] + 16) >> 5 : ref[b + idx + 1];
            pred[y * N + x] = v;
        }
    if (cidx == 0 && N < 32) {
        if (mode == 26)
            for (int y = 0; y < N; ++y) pred[y * N] = clip255(top[1] + ((left[1 + y] - left[0]) >> 1));
        else if (mode == 10)
            for (int x = 0; x < N; ++x) pred[x] = clip255(left[1] + ((top[1 + x] - top[0]) >> 1));
    }
}

// Intra modes whose N x N prediction never reads the below-left references p[-1][N .. 2N-1] (not
// even through the [1 2 1] reference filter), bit m = mode m, for luma (cidx 0) or chroma.  The
// first unit of a CTB has its below-left neighbour (the left CTB's last unit) available to the
// decoder but not yet reconstructed by the encoder's raster wavefront; it restricts itself to
// these modes and predicts with the below-left treated as unavailable -- for these modes the
// same samples as the decoder's.  Found by perturbing the below-left samples.
inline uint64_t bl_safe_modes(int log2n, int cidx) {
    const int N = 1 << log2n;
    int L[65], T[65], L2[65], p0[32 * 32], p1[32 * 32], p2[32 * 32];
    for (int k = 0; k <= 2 * N; ++k) {
        L[k] = (k * 37 + 11) & 255;
        T[k] = (k * 53 + 7) & 255;
    }
    uint64_t m = 0;
    for (int mode = 0; mode < 35; ++mode) {
        intra_predict(mode, log2n, cidx, L, T, p0);
        bool same = true;
        for (int v = 1; v <= 2 && same; ++v) {
            for (int k = 0; k <= 2 * N; ++k) L2[k] = k > N ? (L[k] + 97 * v) & 255 : L[k];
            intra_predict(mode, log2n, cidx, L2, T, v == 1 ? p1 : p2);
            for (int i = 0; i < N * N; ++i) same = same && (v == 1 ? p1[i] : p2[i]) == p0[i];
        }
        if (same) m |= 1ull << mode;
    }
    return m;
}

// Most probable modes (8.4.2) from the left / above candidates (the above one only inside the CTB).
MXHD void mpm_list(int cand_a, int cand_b, int* l) {
    if (cand_a == cand_b) {
        if (cand_a < 2) {
            l[0] = 0;
            l[1] = 1;
            l[2] = 26;
        } else {
            l[0] = cand_a;
            l[1] = 2 + ((cand_a + 29) % 32);
            l[2] = 2 + ((cand_a - 2 + 1) % 32);
        }
    } else {
        l[0] = cand_a;
        l[1] = cand_b;
        if (cand_a != 0 && cand_b != 0)
            l[2] = 0;
        else if (cand_a != 1 && cand_b != 1)
            l[2] = 1;
        else
            l[2] = 26;
    }
}

// ---------------------------------------------------------------- inter interpolation (8.5.3.3.3)
constexpr int8_t kLumaTap[4][8] = {
    {0, 0, 0, 64, 0, 0, 0, 0}, {-1, 4, -10, 58, 17, -5, 1, 0}, {-1, 4, -11, 40, 40, -11, 4, -1}, {0, 1, -5, 17, 58, -10, 4, -1}};
constexpr int8_t kChromaTap[8][4] = {{0, 64, 0, 0},     {-2, 58, 10, -2}, {-4, 54, 16, -2}, {-6, 46, 28, -4},
                                     {-4, 36, 36, -4},  {-4, 28, 46, -6}, {-2, 16, 54, -4}, {-2, 10, 58, -2}};

MXHD int ref_at(const uint8_t* p, int pitch, int w, int h, int x, int y, int step = 1) {
    x = x < 0 ? 0 : (x >= w ? w - 1 : x);
    y = y < 0 ? 0 : (y >= h ? h - 1 : y);
    return p[y * pitch + x * step];
}

// Uni-predicted luma sample at integer position (x, y) displaced by the quarter-pel
// vector (mvx, mvy); reference plane w x h with edge clamping.
MXHD int luma_mc(const uint8_t* ref, int pitch, int w, int h, int x, int y, int mvx, int mvy) {
    const int xi = x + (mvx >> 2), yi = y + (mvy >> 2), fx = mvx & 3, fy = mvy & 3;
    int v;
    if (!fx && !fy) {
        v = ref_at(ref, pitch, w, h, xi, yi) << 6;
    } else if (!fy) {
        v = 0;
        for (int i = 0; i < 8; ++i) v += kLumaTap[fx][i] * ref_at(ref, pitch, w, h, xi + i - 3, yi);
    } else if (!fx) {
        v = 0;
        for (int i = 0; i < 8; ++i) v += kLumaTap[fy][i] * ref_at(ref, pitch, w, h, xi, yi + i - 3);
    } else {
        int s = 0;
        for (int n = 0; n < 8; ++n) {
            int t = 0;
            for (int i = 0; i < 8; ++i) t += kLumaTap[fx][i] * ref_at(ref, pitch, w, h, xi + i - 3, yi + n - 3);
            s += kLumaTap[fy][n] * t;
        }
        v = s >> 6;
    }
    return clip255((v + 32) >> 6);
}

// Chroma sample (interleaved NV12 plane, comp 0 = Cb, 1 = Cr) at chroma position (x, y),
// luma quarter-pel vector = chroma eighth-pel vector for 4:2:0.
MXHD int chroma_mc(const uint8_t* uv, int pitch, int cw, int ch, int comp, int x, int y, int mvx, int mvy) {
    const int xi = x + (mvx >> 3), yi = y + (mvy >> 3), fx = mvx & 7, fy = mvy & 7;
    const uint8_t* p = uv + comp;
    int v;
    if (!fx && !fy) {
        v = ref_at(p, pitch, cw, ch, xi, yi, 2) << 6;
    } else if (!fy) {
        v = 0;
        for (int i = 0; i < 4; ++i) v += kChromaTap[fx][i] * ref_at(p, pitch, cw, ch, xi + i - 1, yi, 2);
    } else if (!fx) {
        v = 0;
        for (int i = 0; i < 4; ++i) v += kChromaTap[fy][i] * ref_at(p, pitch, cw, ch, xi, yi + i - 1, 2);
    } else {
        int s = 0;
        for (int n = 0; n < 4; ++n) {
            int t = 0;
            for (int i = 0; i < 4; ++i) t += kChromaTap[fx][i] * ref_at(p, pitch, cw, ch, xi + i - 1, yi + n - 1, 2);
            s += kChromaTap[fy][n] * t;
        }
        v = s >> 6;
    }
    return clip255((v + 32) >> 6);
}

// ---------------------------------------------------------------- CABAC (9.3)
constexpr uint8_t kLps[64][4] = {
    {128, 176, 208, 240}, {128, 167, 197, 227}, {128, 158, 187, 216}, {123, 150, 178, 205}, {116, 142, 169, 195},
    {111, 135, 160, 185}, {105, 128, 152, 175}, {100, 122, 144, 166}, {95, 116, 137, 158},  {90, 110, 130, 150},
    {85, 104, 123, 142},  {81, 99, 117, 135},   {77, 94, 111, 128},   {73, 89, 105, 122},   {69, 85, 100, 116},
    {66, 80, 95, 110},    {62, 76, 90, 104},    {59, 72, 86, 99},     {56, 69, 81, 94},     {53, 65, 77, 89},
    {51, 62, 73, 85},     {48, 59, 69, 80},     {46, 56, 66, 76},     {43, 53, 63, 72},     {41, 50, 59, 69},
    {39, 48, 56, 65},     {37, 45, 54, 62},     {35, 43, 51, 59},     {33, 41, 48, 56},     {32, 39, 46, 53},
    {30, 37, 43, 50},     {29, 35, 41, 48},     {27, 33, 39, 45},     {26, 31, 37, 43},     {24, 30, 35, 41},
    {23, 28, 33, 39},     {22, 27, 32, 37},     {21, 26, 30, 35},     {20, 24, 29, 33},     {19, 23, 27, 31},
    {18, 22, 26, 30},     {17, 21, 25, 28},     {16, 20, 23, 27},     {15, 19, 22, 25},     {14, 18, 21, 24},
    {14, 17, 20, 23},     {13, 16, 19, 22},     {12, 15, 18, 21},     {12, 14, 17, 20},     {11, 14, 16, 19},
    {11, 13, 15, 18},     {10, 12, 15, 17},     {10, 12, 14, 16},     {9, 11, 13, 15},      {9, 11, 12, 14},
    {8, 10, 12, 14},      {8, 9, 11, 13},       {7, 9, 11, 12},       {7, 9, 10, 12},       {7, 8, 10, 11},
    {6, 8, 9, 11},        {6, 7, 9, 10},        {6, 7, 8, 9},         {2, 2, 2, 2}};
constexpr uint8_t kNextLps[64] = {0,  0,  1,  2,  2,  4,  4,  5,  6,  7,  8,  9,  9,  11, 11, 12,
                                  13, 13, 15, 15, 16, 16, 18, 18, 19, 19, 21, 21, 22, 22, 23, 24,
                                  24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30, 31, 32, 32, 33,
                                  33, 33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63};

// Context index layout (this encoder's numbering; the decoder uses the same initValues)
enum Ctx : int {
    C_SKIP = 0,            // 3
    C_MERGE_FLAG = 3,      // 1
    C_MERGE_IDX = 4,       // 1
    C_PRED_MODE = 5,       // 1
    C_PART_MODE = 6,       // 4
    C_PREV_INTRA = 10,     // 1
    C_CHROMA_PRED = 11,    // 1
    C_RQT_ROOT = 12,       // 1
    C_MVP = 13,            // 1
    C_MVD_G0 = 14,         // 1
    C_MVD_G1 = 15,         // 1
    C_CBF_LUMA = 16,       // 2
    C_CBF_CHROMA = 18,     // 4
    C_QP_DELTA = 22,       // 2
    C_LAST_X = 24,         // 18
    C_LAST_Y = 42,         // 18
    C_CSBF = 60,           // 4
    C_SIG = 64,            // 42
    C_GT1 = 106,           // 24
    C_GT2 = 130,           // 6
    C_SPLIT_TRANSFORM = 136,  // 3
    C_SPLIT_CU = 139,      // 3
    C_SAO_MERGE = 142,     // 1 (sao_merge_left_flag and sao_merge_up_flag)
    C_SAO_TYPE = 143,      // 1 (first bin of sao_type_idx_luma / _chroma)
    C_NUM = 144
};

// initValue per initType (0: I, 1: P without cabac_init_flag, 2: B), Tables 9-5..9-37
constexpr uint8_t kCtxInit[3][C_NUM] = {
    {// I
     154, 154, 154,                          // skip (unused)
     154, 154, 154,                          // merge flag / idx, pred mode (unused)
     184, 154, 154, 154,                     // part_mode
     184, 63, 154, 154, 154, 154,            // prev_intra, chroma_pred, rqt_root, mvp, mvd g0/g1 (unused)
     111, 141,                               // cbf_luma
     94, 138, 182, 154,                      // cbf_cb/cr
     154, 154,                               // cu_qp_delta_abs
     110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,
     110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,
     91, 171, 134, 141,
     111, 111, 125, 110, 110, 94, 124, 108, 124, 107, 125, 141, 179, 153, 125, 107, 125, 141, 179, 153, 125,
     107, 125, 141, 179, 153, 125, 140, 139, 182, 182, 152, 136, 152, 136, 153, 136, 139, 111, 136, 139, 111,
     140, 92, 137, 138, 140, 152, 138, 139, 153, 74, 149, 92, 139, 107, 122, 152, 140, 179, 166, 182, 140, 227,
     122, 197,
     138, 153, 136, 167, 152, 152,
     153, 138, 138,
     139, 141, 157,
     153, 200},
    {// P (initType 1)
     197, 185, 201,
     110, 122, 149,
     154, 139, 154, 154,
     154, 152, 79, 168, 140, 198,
     153, 111,
     149, 107, 167, 154,
     154, 154,
     125, 110, 94, 110, 95, 79, 125, 111, 110, 78, 110, 111, 111, 95, 94, 108, 123, 108,
     125, 110, 94, 110, 95, 79, 125, 111, 110, 78, 110, 111, 111, 95, 94, 108, 123, 108,
     121, 140, 61, 154,
     155, 154, 139, 153, 139, 123, 123, 63, 153, 166, 183, 140, 136, 153, 154, 166, 183, 140, 136, 153, 154,
     166, 183, 140, 136, 153, 154, 170, 153, 123, 123, 107, 121, 107, 121, 167, 151, 183, 140, 151, 183, 140,
     154, 196, 196, 167, 154, 152, 167, 182, 182, 134, 149, 136, 153, 121, 136, 137, 169, 194, 166, 167, 154, 167,
     137, 182,
     107, 167, 91, 122, 107, 167,
     124, 138, 94,
     107, 139, 126,
     153, 185},
    {// B (initType 2)
     197, 185, 201,
     154, 137, 134,
     154, 139, 154, 154,
     183, 152, 79, 168, 169, 198,
     153, 111,
     149, 92, 167, 154,
     154, 154,
     125, 110, 124, 110, 95, 94, 125, 111, 111, 79, 125, 126, 111, 111, 79, 108, 123, 93,
     125, 110, 124, 110, 95, 94, 125, 111, 111, 79, 125, 126, 111, 111, 79, 108, 123, 93,
     121, 140, 61, 154,
     170, 154, 139, 153, 139, 123, 123, 63, 124, 166, 183, 140, 136, 153, 154, 166, 183, 140, 136, 153, 154,
     166, 183, 140, 136, 153, 154, 170, 153, 138, 138, 122, 121, 122, 121, 167, 151, 183, 140, 151, 183, 140,
     154, 196, 167, 167, 154, 152, 167, 182, 182, 134, 149, 136, 153, 121, 136, 122, 169, 208, 166, 167, 154, 152,
     167, 182,
     107, 167, 91, 107, 107, 167,
     224, 167, 122,
     107, 139, 126,
     153, 160}};

// Context state byte: (pStateIdx << 1) | valMps (9.3.2.2)
MXHD uint8_t ctx_init_state(int init_value, int qp) {
    const int slope = (init_value >> 4) * 5 - 45;
    const int offset = ((init_value & 15) << 3) - 16;
    qp = qp < 0 ? 0 : (qp > 51 ? 51 : qp);
    int pre = ((slope * qp) >> 4) + offset;
    pre = pre < 1 ? 1 : (pre > 126 ? 126 : pre);
    return pre <= 63 ? (uint8_t)((63 - pre) << 1) : (uint8_t)(((pre - 64) << 1) | 1);
}
MXHD void ctx_init_all(uint8_t* ctx, int init_type, int qp) {
    for (int i = 0; i < C_NUM; ++i) ctx[i] = ctx_init_state(kCtxInit[init_type][i], qp);
}

// Context states in a byte array (host encoder; any memory on the device).
// A context store also provides the state-transition tables (rangeTabLps, transIdxLps).
struct ArrCtx {
    uint8_t* p;
    MXHD uint32_t get(int i) const { return p[i]; }
    MXHD void set(int i, uint32_t v) { p[i] = (uint8_t)v; }
    MXHD uint32_t lps(uint32_t s, uint32_t q) const { return kLps[s][q]; }
    MXHD uint32_t next_lps(uint32_t s) const { return kNextLps[s]; }
};

// Wave-uniform value hint: on the device the CABAC kernel runs one slice per wave with every
// lane holding the same coder state; readfirstlane keeps that state in SGPRs (the compiler
// cannot prove uniformity through the coder's data-dependent branches).
MXHD uint32_t uni(uint32_t v) {
#ifdef __HIP_DEVICE_COMPILE__
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
#else
    return v;
#endif
}
MXHD int uni(int v) { return (int)uni((uint32_t)v); }

// Arithmetic encoder (HM-style: 32-bit low register, byte output with carry resolution).
struct CabacEnc {
    uint32_t low, range;
    int bits_left, buffered, num_buffered;
    uint8_t* out;
    uint32_t pos, cap, overflow;

    MXHD void start(uint8_t* o, uint32_t c) {
        low = 0;
        range = 510;
        bits_left = 23;
        buffered = 0xff;
        num_buffered = 0;
        out = o;
        pos = 0;
        cap = c;
        overflow = 0;
    }
    MXHD void put_byte(uint32_t b) {
        if (pos < cap)
            out[pos] = (uint8_t)b;
        else
            overflow = 1;
        pos = uni(pos + 1);
    }
    MXHD void write_out() {
        const uint32_t lead = uni(low >> (24 - bits_left));
        bits_left += 8;
        low &= 0xffffffffu >> bits_left;
        num_buffered = uni(num_buffered);
        buffered = uni(buffered);
        if (lead == 0xff) {
            ++num_buffered;
        } else if (num_buffered > 0) {
            const uint32_t carry = lead >> 8;
            put_byte(buffered + carry);
            buffered = (int)(lead & 0xff);
            const uint32_t fill = (0xff + carry) & 0xff;
            while (num_buffered > 1) {
                put_byte(fill);
                --num_buffered;
            }
        } else {
            num_buffered = 1;
            buffered = (int)lead;
        }
    }
    MXHD void test_write_out() {
        low = uni(low);
        range = uni(range);
        bits_left = uni(bits_left);
        if (bits_left < 12) write_out();
    }
    // Context-coded bin; Ctx stores the 142 state bytes ((pStateIdx << 1) | valMps).
    template <class Ctx>
    MXHD void bin(Ctx& cx, int idx, int b) {
        const uint32_t st = cx.get(idx);
        uint32_t s = st >> 1, mps = st & 1;
        const uint32_t lps = cx.lps(s, (range >> 6) & 3);
        range -= lps;
        if ((uint32_t)b != mps) {
            const int nb = __builtin_clz(lps) - 23;
            low = (low + range) << nb;
            range = lps << nb;
            if (s == 0) mps ^= 1;
            s = cx.next_lps(s);
            bits_left -= nb;
            cx.set(idx, (s << 1) | mps);
            test_write_out();
        } else {
            s = s < 62 ? s + 1 : s;
            cx.set(idx, (s << 1) | mps);
            range = uni(range);
            if (range >= 256) return;
            low <<= 1;
            range <<= 1;
            --bits_left;
            test_write_out();
        }
    }
    MXHD void bypass(int b) {
        low <<= 1;
        if (b) low += range;
        --bits_left;
        test_write_out();
    }
    // n bypass bins at once (MSB first): low = (low << n) + range * v, in chunks of 8 so the
    // 32-bit register never overflows (HM encodeBinsEP)
    MXHD void bypass_bits(uint32_t v, int n) {
        while (n > 8) {
            n -= 8;
            low = (low << 8) + range * ((v >> n) & 0xffu);
            bits_left -= 8;
            test_write_out();
        }
        if (n > 0) {
            low = (low << n) + range * (v & ((1u << n) - 1));
            bits_left -= n;
            test_write_out();
        }
    }
    MXHD void terminate(int b) {
        range -= 2;
        if (b) {
            low += range;
            low <<= 7;
            range = 2 << 7;
            bits_left -= 7;
        } else if (range >= 256) {
            return;
        } else {
            low <<= 1;
            range <<= 1;
            --bits_left;
        }
        test_write_out();
    }
    // Flush after the final terminate(1) and append rbsp_slice_segment_trailing_bits.
    MXHD void flush() {}  // (BinRec interface: nothing buffered here)
    MXHD void finish_slice() {
        if (low >> (32 - bits_left)) {
            put_byte(buffered + 1);
            while (num_buffered > 1) {
                put_byte(0x00);
                --num_buffered;
            }
            low -= 1u << (32 - bits_left);
        } else {
            if (num_buffered > 0) put_byte(buffered);
            while (num_buffered > 1) {
                put_byte(0xff);
                --num_buffered;
            }
        }
        // remaining (24 - bits_left) bits of low >> 8, then the stop bit, then zero alignment
        int n = 24 - bits_left;
        uint32_t v = (low >> 8) & ((1u << n) - 1);
        v = (v << 1) | 1;
        ++n;
        const int pad = (8 - (n & 7)) & 7;
        v <<= pad;
        n += pad;
        for (int i = n - 8; i >= 0; i -= 8) put_byte((v >> i) & 0xff);
    }
};

// k-th order Exp-Golomb, bypass coded (9.3.3.3): m ones, a zero, then k + m suffix bits.  E is
// the arithmetic coder (CabacEnc) or the bin recorder (BinRec) -- the syntax coders below are
// templates over both.
template <class E>
MXHD void code_egk(E& e, uint32_t v, int k) {
    int m = 0;
    while (v >= (1u << k)) {
        v -= 1u << k;
        ++k;
        ++m;
    }
    e.bypass_bits((1u << m) - 1, m);
    e.bypass_bits(v, k + 1);  // leading zero + k bits
}

// ---------------------------------------------------------------- CU description
enum CuType : uint8_t { kCuSkip = 0, kCuMerge = 1, kCuAmvp = 2, kCuIntra = 3 };

struct CuInfo {
    uint8_t type;        // CuType
    uint8_t intra_mode;  // luma intra mode (chroma uses mode 4 = DM)
    uint8_t qp;          // QP the residual was quantised with
    uint8_t cbf;         // bit0 Y, bit1 Cb, bit2 Cr
    int16_t mvx, mvy;    // final quarter-pel motion vector
    int16_t mvdx, mvdy;  // AMVP motion vector difference
    uint8_t mvp_idx;
    uint8_t last[3];     // last significant scan index per TU (Y 0..255, Cb/Cr 0..63)
    uint16_t csbf_y;     // coded sub-block mask (bit = sub-block scan index)
    uint8_t csbf_c[2];
    // transform tree of inter CUs: 0 = not coded (SPS depth 0), 1 = one 16x16 TU, 2 = split into
    // four 8x8 luma TUs (sub-blocks 4k..4k+3) and 4x4 chroma TUs (Cb sub-block 16+k, Cr 20+k)
    uint8_t tu_split;
    uint8_t cbf_y4;  // split: bit k = luma TU k coded
    uint8_t cbf_c4;  // split: bit k = Cb TU k, bit 4+k = Cr TU k coded
    uint8_t est_bytes;  // entropy-coder work estimate of a coded CU: cu_bits_est / 8, capped 255 (set_est_bytes)
    // coding-tree depth of this 16x16 unit: 0 = one of the four units of a CU32 (type, vector, QP
    // and mvp / mvd equal in all four; the CU's prediction syntax lives in the z-order first unit),
    // 1 = a CU16
    uint8_t ct;
    // split transform tree (tu_split 2): bit k = the 8x8 luma node k split again into four 4x4
    // luma TUs (sub-blocks 4k + j, z order; its chroma stays one 4x4 TU per component), and the
    // coded flags of those 4x4 TUs (bit 4k + j)
    uint8_t tu4;
    uint16_t cbf_y16;
    uint8_t rsv[4];
};
static_assert(sizeof(CuInfo) == 32, "CuInfo layout");
constexpr int kCuWords = (int)(sizeof(CuInfo) / 4);

// Per-TU summary (cbf, last position, coded sub-blocks) of coefficients in scan order.
MXHD bool tu_summary(const int16_t* c, int n, uint8_t* last, uint32_t* csbf) {
    int l = -1;
    uint32_t m = 0;
    for (int i = 0; i < n; ++i)
        if (c[i]) {
            l = i;
            m |= 1u << (i >> 4);
        }
    *last = (uint8_t)(l < 0 ? 0 : l);
    *csbf = m;
    return l >= 0;
}

// CU summary from its levels (cbf bits, per-TU last positions and coded sub-blocks).  For a
// split transform tree the per-TU cbf go to cbf_y4 / cbf_c4, and last[] / csbf_* hold sums
// and unions that only feed the entropy-cost estimate (code_cu recomputes per-TU values).
MXHD void cu_summarise(CuInfo& c, const int16_t* co) {
    uint32_t m;
    c.cbf = 0;
    c.cbf_y4 = c.cbf_c4 = 0;
    if (c.tu_split != 2) {
        c.tu4 = 0;
        c.cbf_y16 = 0;
        if (tu_summary(co, 256, &c.last[0], &m)) c.cbf |= 1;
        c.csbf_y = (uint16_t)m;
        if (tu_summary(co + 256, 64, &c.last[1], &m)) c.cbf |= 2;
        c.csbf_c[0] = (uint8_t)m;
        if (tu_summary(co + 320, 64, &c.last[2], &m)) c.cbf |= 4;
        c.csbf_c[1] = (uint8_t)m;
        return;
    }
    uint32_t lsum = 0, csy = 0;
    c.cbf_y16 = 0;
    for (int k = 0; k < 4; ++k) {
        uint8_t l;
        if ((c.tu4 >> k) & 1) {  // four 4x4 TUs (one sub-block each)
            for (int j = 0; j < 4; ++j)
                if (tu_summary(co + 64 * k + 16 * j, 16, &l, &m)) {
                    c.cbf_y16 |= (uint16_t)(1u << (4 * k + j));
                    c.cbf_y4 |= (uint8_t)(1u << k);
                    lsum += l + 1u;
                    csy |= 1u << (4 * k + j);
                }
        } else if (tu_summary(co + 64 * k, 64, &l, &m)) {
            c.cbf_y4 |= (uint8_t)(1u << k);
            lsum += l + 1u;
            csy |= m << (4 * k);
        }
    }
    c.cbf |= c.cbf_y4 ? 1 : 0;
    c.last[0] = (uint8_t)(lsum ? (lsum > 256 ? 255 : lsum - 1) : 0);
    c.csbf_y = (uint16_t)csy;
    for (int comp = 0; comp < 2; ++comp) {
        uint32_t csum = 0, cm = 0;
        for (int k = 0; k < 4; ++k) {
            uint8_t l;
            if (tu_summary(co + 256 + 64 * comp + 16 * k, 16, &l, &m)) {
                c.cbf_c4 |= (uint8_t)(1u << (4 * comp + k));
                csum += l + 1u;
                cm |= 1u << k;
            }
        }
        if (cm) c.cbf |= (uint8_t)(2 << comp);
        c.last[1 + comp] = (uint8_t)(csum ? csum - 1 : 0);
        c.csbf_c[comp] = (uint8_t)cm;
    }
}

// ---------------------------------------------------------------- residual_coding (7.3.8.11)
// last_sig_coeff prefix group of a position and the smallest position of a group
MXHD int last_group(int pos) {
    if (pos < 4) return pos;
    const int l = 31 - __builtin_clz((uint32_t)pos);
    return 2 * l + ((pos >> (l - 1)) & 1);
}
MXHD int last_min(int g) { return g < 4 ? g : (1 << ((g >> 1) - 1)) * (2 + (g & 1)); }

template <class E, class Ctx>
MXHD void code_last_prefix(E& e, Ctx& ctx, int base, int pos, int log2n, int cidx) {
    const int off = cidx ? 15 : 3 * (log2n - 2) + ((log2n - 1) >> 2);
    const int shift = cidx ? log2n - 2 : (log2n + 1) >> 2;
    const int prefix = last_group(pos);
    const int cmax = (log2n << 1) - 1;
    for (int b = 0; b < prefix; ++b) e.bin(ctx, base + off + (b >> shift), 1);
    if (prefix < cmax) e.bin(ctx, base + off + (prefix >> shift), 0);
}
template <class E>
MXHD void code_last_suffix(E& e, int pos) {
    const int prefix = last_group(pos);
    if (prefix > 3) e.bypass_bits((uint32_t)(pos - last_min(prefix)), (prefix >> 1) - 1);
}

// coeff_abs_level_remaining (9.3.3.11)
template <class E>
MXHD void code_remaining(E& e, uint32_t v, int rice) {
    if (v < (4u << rice)) {
        const uint32_t pre = v >> rice;  // pre ones, a zero, rice LSBs
        e.bypass_bits((((1u << pre) - 1) << (rice + 1)) | (v & ((1u << rice) - 1)), (int)pre + 1 + rice);
    } else {
        e.bypass_bits(15, 4);
        code_egk(e, v - (4u << rice), rice + 1);
    }
}

// Coefficient access for the residual coder.  A CU's 24 coded sub-blocks are numbered
// luma 0..15, Cb 16..19, Cr 20..23 (each TU in scan order); sig(sb) / neg(sb) are 16-bit masks
// (bit n = scan position n) and absval(sb * 16 + n) the level magnitude.
struct CoefArray {  // host / generic: the CU's 384 int16 levels
    const int16_t* c;
    MXHD uint32_t sig(int sb) const {
        uint32_t m = 0;
        for (int n = 0; n < 16; ++n) m |= (c[sb * 16 + n] != 0 ? 1u : 0u) << n;
        return m;
    }
    MXHD uint32_t neg(int sb) const {
        uint32_t m = 0;
        for (int n = 0; n < 16; ++n) m |= (c[sb * 16 + n] < 0 ? 1u : 0u) << n;
        return m;
    }
    MXHD int absval(int i) const { return c[i] < 0 ? -c[i] : c[i]; }
};

MXHD int msb16(uint32_t m) { return 31 - __builtin_clz(m); }  // m != 0

// sigCtx of a 4x4 TU position (raster y*4+x), 9.3.4.2.5
constexpr uint8_t kCtxIdxMap4x4[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};

// last significant scan index and coded-sub-block mask of a TU of `nsb` sub-blocks (1 or 4)
// starting at CU sub-block sb0, from the coefficient accessor's significance masks
template <class Cf>
MXHD int tu_last(const Cf& cf, int sb0, int nsb, uint32_t* csbf) {
    int last = -1;
    uint32_t m = 0;
    for (int i = 0; i < nsb; ++i) {
        const uint32_t sg = cf.sig(sb0 + i);
        if (sg) {
            m |= 1u << i;
            last = i * 16 + msb16(sg);
        }
    }
    *csbf = m;
    return last;
}

// One TU of a CU for the residual coder: size 2^log2n (4, 8 or 16; scanIdx 0), sub-blocks from
// CU sub-block sb0, last significant scan index, coded sub-blocks (bit = scan index in the TU).
struct TuDesc {
    int sb0, log2n, cidx, last_idx;
    uint32_t csbf_mask;
    int scan;  // scanIdx (intra_scan_idx for intra 4x4 / 8x8 luma and 4x4 chroma TUs, else 0)
};
// coded (or inferred: DC and last) sub-blocks of a TU as a raster mask
MXHD uint32_t tu_csbf_raster(const TuDesc& t) {
    const int last_sb = t.last_idx >> 4, sbw = 1 << (t.log2n - 2);
    uint32_t r = 0;
    for (int i = 0; i <= last_sb; ++i) {
        int sx, sy;
        sb_grid_pos(t.log2n, t.scan, i, &sx, &sy);
        if (i == 0 || i == last_sb || ((t.csbf_mask >> i) & 1)) r |= 1u << (sy * sbw + sx);
    }
    return r;
}

// last_sig_coeff_x / _y prefix and suffix of a TU (the vertical scan codes the pair swapped)
template <class E, class Ctx>
MXHD void code_tu_last(E& e, Ctx& ctx, const TuDesc& t) {
    int lx, ly;
    if (t.scan == 2)
        scan_pos_s(t.log2n, t.scan, t.last_idx, &ly, &lx);
    else
        scan_pos_s(t.log2n, t.scan, t.last_idx, &lx, &ly);
    code_last_prefix(e, ctx, C_LAST_X, lx, t.log2n, t.cidx);
    code_last_prefix(e, ctx, C_LAST_Y, ly, t.log2n, t.cidx);
    code_last_suffix(e, lx);
    code_last_suffix(e, ly);
}

// greater1Ctx after a sub-block with levels is 0 iff one of its first 8 coded levels (scan
// positions high to low) exceeds 1: the next coded sub-block of the TU then uses ctxSet + 1.
template <class Cf>
MXHD bool sb_any_gt1(const Cf& cf, int sb, uint32_t sig) {
    int k = 0;
    for (uint32_t m = sig; m && k < 8; ++k) {
        const int n = msb16(m);
        m &= ~(1u << n);
        if (cf.absval(sb * 16 + n) > 1) return true;
    }
    return false;
}

// Sub-block i of TU t (coded_sub_block_flag, significance, greater1 / greater2, signs, remaining
// levels).  csbf_r: tu_csbf_raster(t).  prev_gt1: for the previous sub-block with levels in this
// TU (coding order), whether it had a greater1 flag set (sb_any_gt1); -1: none.  Every sub-block
// of a TU is independent given these, so the GPU binarises them in parallel.
template <class E, class Ctx, class Cf>
MXHD void code_sub_block(E& e, Ctx& ctx, const Cf& cf, const TuDesc& t, uint32_t csbf_r, int i, int prev_gt1) {
    const int log2n = t.log2n, cidx = t.cidx;
    const int last_sb = t.last_idx >> 4, last_n = t.last_idx & 15;
    const int sbw = 1 << (log2n - 2);
    int sx, sy;
    sb_grid_pos(log2n, t.scan, i, &sx, &sy);
    const bool right = sx + 1 < sbw && ((csbf_r >> (sy * sbw + sx + 1)) & 1);
    const bool below = sy + 1 < sbw && ((csbf_r >> ((sy + 1) * sbw + sx)) & 1);
    bool infer_dc = false;
    if (i < last_sb && i > 0) {
        const int coded = (t.csbf_mask >> i) & 1;
        e.bin(ctx, C_CSBF + (cidx ? 2 : 0) + ((right || below) ? 1 : 0), coded);
        if (!coded) return;
        infer_dc = true;
    }
    const uint32_t sig = cf.sig(t.sb0 + i);
    // significance
    const int prev_csbf = (right ? 1 : 0) | (below ? 2 : 0);
    const int nstart = (i == last_sb) ? last_n - 1 : 15;
    for (int n = nstart; n >= 0; --n) {
        if (n == 0 && infer_dc) break;
        const int bit = (sig >> n) & 1;
        int xp, yp;
        sb_pos(t.scan, n, &xp, &yp);
        int sc;
        if (log2n == 2) {
            sc = kCtxIdxMap4x4[(yp << 2) + xp];
        } else if (i == 0 && n == 0) {
            sc = 0;
        } else {
            if (prev_csbf == 0)
                sc = (xp + yp == 0) ? 2 : (xp + yp < 3 ? 1 : 0);
            else if (prev_csbf == 1)
                sc = yp == 0 ? 2 : (yp == 1 ? 1 : 0);
            else if (prev_csbf == 2)
                sc = xp == 0 ? 2 : (xp == 1 ? 1 : 0);
            else
                sc = 2;
            if (cidx == 0) {
                if (i > 0) sc += 3;
                sc += log2n == 3 ? (t.scan == 0 ? 9 : 15) : 21;
            } else {
                sc += log2n == 3 ? 9 : 12;
            }
        }
        e.bin(ctx, C_SIG + (cidx ? 27 : 0) + sc, bit);
        if (bit) infer_dc = false;
    }
    if (!sig) return;
    // levels of the nonzero coefficients, n = 15 down to 0 (greater1 flags for the first 8)
    const int base_i = (t.sb0 + i) * 16;
    int ctx_set = (i == 0 || cidx > 0) ? 0 : 2;
    if (prev_gt1 == 1) ++ctx_set;
    int g1ctx = 1, g2_pos = -1, k = 0;
    for (uint32_t m = sig; m && k < 8; ++k) {
        const int n = msb16(m);
        m &= ~(1u << n);
        const int g1 = cf.absval(base_i + n) > 1 ? 1 : 0;
        e.bin(ctx, C_GT1 + (cidx ? 16 : 0) + ctx_set * 4 + (g1ctx < 3 ? g1ctx : 3), g1);
        if (g1) {
            g1ctx = 0;
            if (g2_pos < 0) g2_pos = n;
        } else if (g1ctx > 0) {
            ++g1ctx;
        }
    }
    if (g2_pos >= 0) e.bin(ctx, C_GT2 + (cidx ? 4 : 0) + ctx_set, cf.absval(base_i + g2_pos) > 2);
    {  // sign bits of the nonzero levels, n = 15 down to 0, as one bypass run
        const uint32_t neg = cf.neg(t.sb0 + i);
        uint32_t bits = 0;
        int nb = 0;
        for (uint32_t m = sig; m; ++nb) {
            const int n = msb16(m);
            m &= ~(1u << n);
            bits = (bits << 1) | ((neg >> n) & 1);
        }
        e.bypass_bits(bits, nb);
    }
    int rice = 0;
    k = 0;
    for (uint32_t m = sig; m; ++k) {
        const int n = msb16(m);
        m &= ~(1u << n);
        if (k < 8 && n != g2_pos && g2_pos < 0) continue;  // all levels 1: nothing left to code
        const int a = cf.absval(base_i + n);
        int base, thr;
        if (k < 8) {
            base = 1 + (a > 1 ? 1 : 0) + (n == g2_pos && a > 2 ? 1 : 0);
            thr = (n == g2_pos) ? 3 : 2;
        } else {
            base = 1;
            thr = 1;
        }
        if (base == thr) {
            code_remaining(e, (uint32_t)(a - base), rice);
            if (a > 3 * (1 << rice)) rice = rice + 1 < 4 ? rice + 1 : 4;
        }
    }
}

// One TU: last position, then its sub-blocks from the last one down to the DC sub-block.
template <class E, class Ctx, class Cf>
MXHD void code_residual(E& e, Ctx& ctx, const Cf& cf, const TuDesc& t) {
    code_tu_last(e, ctx, t);
    const uint32_t csbf_r = tu_csbf_raster(t);
    int prev_gt1 = -1;
    for (int i = t.last_idx >> 4; i >= 0; --i) {
        code_sub_block(e, ctx, cf, t, csbf_r, i, prev_gt1);
        const uint32_t sig = cf.sig(t.sb0 + i);
        if (sig && (i == 0 || i == (t.last_idx >> 4) || ((t.csbf_mask >> i) & 1)))
            prev_gt1 = sb_any_gt1(cf, t.sb0 + i, sig) ? 1 : 0;
    }
}

// ---------------------------------------------------------------- CU syntax (7.3.8.5)
template <class E, class Ctx>
MXHD void code_mvd(E& e, Ctx& ctx, int dx, int dy) {
    const int ax = dx < 0 ? -dx : dx, ay = dy < 0 ? -dy : dy;
    e.bin(ctx, C_MVD_G0, ax > 0);
    e.bin(ctx, C_MVD_G0, ay > 0);
    if (ax > 0) e.bin(ctx, C_MVD_G1, ax > 1);
    if (ay > 0) e.bin(ctx, C_MVD_G1, ay > 1);
    if (ax > 0) {
        if (ax > 1) code_egk(e, (uint32_t)(ax - 2), 1);
        e.bypass(dx < 0);
    }
    if (ay > 0) {
        if (ay > 1) code_egk(e, (uint32_t)(ay - 2), 1);
        e.bypass(dy < 0);
    }
}

MXHD int qp_delta_wrap(int qp, int pred) { return ((qp - pred + 26 + 52) % 52) - 26; }

// cu_qp_delta_abs (TU prefix of 5 context bins + EG0 suffix) and its sign
template <class E, class Ctx>
MXHD void code_qp_delta(E& e, Ctx& ctx, int d) {
    const int a = d < 0 ? -d : d;
    const int pre = a < 5 ? a : 5;
    for (int k = 0; k < pre; ++k) e.bin(ctx, C_QP_DELTA + (k ? 1 : 0), 1);
    if (pre < 5) e.bin(ctx, C_QP_DELTA + (pre ? 1 : 0), 0);
    if (a >= 5) code_egk(e, (uint32_t)(a - 5), 0);
    if (a) e.bypass(d < 0);
}

// sao() syntax of a CTB (defined with SAO below)
template <class E, class Ctx>
MXHD void code_sao_w(E& e, Ctx& ctx, uint32_t p0, uint32_t p1, uint32_t p2, bool has_l, uint32_t l0, uint32_t l1,
                     uint32_t l2, bool has_u, uint32_t u0, uint32_t u1, uint32_t u2);

// ---------------------------------------------------------------- coding tree (7.3.8.2-7.3.8.10)
// The CTB grid over the 16x16 units (mb_w x mb_h units, cw x ch CTBs) and the decoding order:
// CTBs in raster order, the (up to four) units of a CTB in z order.  A unit's *coding position* is
// 4 * ctb + z; positions of units outside the picture stay empty.
MXHD int ctb_cols(int mb_w) { return (mb_w + 1) >> 1; }
MXHD int ctb_rows(int mb_h) { return (mb_h + 1) >> 1; }
MXHD int ctb_of(int x, int y, int cw) { return (y >> 1) * cw + (x >> 1); }
MXHD int cpos_of(int x, int y, int cw) { return (ctb_of(x, y, cw) << 2) | ((y & 1) << 1) | (x & 1); }
MXHD void cpos_xy(int k, int cw, int* x, int* y) {
    const int c = k >> 2;
    *x = ((c % cw) << 1) | (k & 1);
    *y = ((c / cw) << 1) | ((k >> 1) & 1);
}
// CTB c lies entirely inside the picture (its split_cu_flag is coded; else it is inferred 1)
MXHD bool ctb_whole(int c, int cw, int mb_w, int mb_h) {
    return 2 * (c % cw) + 1 < mb_w && 2 * (c / cw) + 1 < mb_h;
}
// z index of the last unit of CTB c inside the picture
MXHD int ctb_last_z(int c, int cw, int mb_w, int mb_h) {
    const bool r = 2 * (c % cw) + 1 < mb_w, b = 2 * (c / cw) + 1 < mb_h;
    return (r && b) ? 3 : (b ? 2 : (r ? 1 : 0));
}

// Neighbour facts of a CU at its origin unit (x, y) for the CU syntax: the units left of and above
// the origin (type -1: not available -- outside the picture or in an earlier slice; every other
// earlier unit precedes in decoding order), their coding-tree depths (split_cu_flag contexts) and
// intra modes for the MPM list (8.4.2: the above unit only counts inside the same CTB, else DC).
struct CuNb {
    int left_type, left_mode, above_type, above_mode, left_ct, above_ct;
};
// get(u): the CuInfo of raster unit u
template <class Get>
MXHD CuNb cu_nb_at(const Get& get, int x, int y, int mb_w, int cw, int first_ctb) {
    CuNb nb{-1, 1, -1, 1, 0, 0};
    if (x > 0 && ctb_of(x - 1, y, cw) >= first_ctb) {
        const CuInfo l = get(y * mb_w + x - 1);
        nb.left_type = l.type;
        nb.left_mode = l.intra_mode;
        nb.left_ct = l.ct;
    }
    if (y > 0 && ctb_of(x, y - 1, cw) >= first_ctb) {
        const CuInfo a = get((y - 1) * mb_w + x);
        nb.above_type = a.type;
        nb.above_mode = (y & 1) ? (int)a.intra_mode : 1;
        nb.above_ct = a.ct;
    }
    return nb;
}
MXHD int mpm_cand_a(const CuNb& nb) { return nb.left_type == kCuIntra ? nb.left_mode : 1; }
MXHD int mpm_cand_b(const CuNb& nb) { return nb.above_type == kCuIntra ? nb.above_mode : 1; }

// merge_idx: truncated rice, cMax MaxNumMergeCand - 1, first bin context coded, rest bypass
template <class E, class Ctx>
MXHD void code_merge_idx(E& e, Ctx& ctx, int idx) {
    e.bin(ctx, C_MERGE_IDX, idx > 0);
    for (int k = 1; k < kMaxMergeCand - 1 && k <= idx; ++k) e.bypass(idx > k);
}

// Prediction syntax of a CU of size 2^log2cb: cu_skip_flag, pred_mode_flag, part_mode (2Nx2N;
// coded for inter CUs and for intra CUs of the minimum size), the intra luma / chroma modes or
// merge_flag / merge_idx / mvd / mvp flag, and rqt_root_cbf (AMVP).  root_cbf: a level is coded
// somewhere in the CU.  Returns whether a transform tree follows (inferred for intra and merge).
template <class E, class Ctx>
MXHD bool code_pred_head(E& e, Ctx& ctx, bool islice, const CuInfo& c, const CuNb& nb, bool root_cbf, int log2cb) {
    if (!islice) {
        const int inc = (nb.left_type == kCuSkip ? 1 : 0) + (nb.above_type == kCuSkip ? 1 : 0);
        e.bin(ctx, C_SKIP + inc, c.type == kCuSkip);
    }
    if (c.type == kCuSkip) {
        code_merge_idx(e, ctx, c.mvp_idx);
        return false;
    }
    const bool intra = c.type == kCuIntra;
    if (!islice) e.bin(ctx, C_PRED_MODE, intra);
    if (!intra || log2cb == kMinCbLog2) e.bin(ctx, C_PART_MODE, 1);  // PART_2Nx2N
    if (intra) {
        int l[3];
        mpm_list(mpm_cand_a(nb), mpm_cand_b(nb), l);
        const int m = c.intra_mode;
        const int hit = (m == l[0]) ? 0 : (m == l[1] ? 1 : (m == l[2] ? 2 : -1));
        e.bin(ctx, C_PREV_INTRA, hit >= 0);
        if (hit >= 0) {
            e.bypass(hit > 0);
            if (hit > 0) e.bypass(hit > 1);
        } else {
            // rem_intra_luma_pred_mode: the mode's rank among the 32 modes outside the list
            int rem = m;
            for (int k = 0; k < 3; ++k) rem -= (l[k] < m) ? 1 : 0;
            e.bypass_bits((uint32_t)rem, 5);
        }
        e.bin(ctx, C_CHROMA_PRED, 0);  // intra_chroma_pred_mode 4 (DM)
        return true;
    }
    const bool merge = c.type == kCuMerge;
    e.bin(ctx, C_MERGE_FLAG, merge);
    if (merge) {
        code_merge_idx(e, ctx, c.mvp_idx);
        return true;
    }
    code_mvd(e, ctx, c.mvdx, c.mvdy);
    e.bin(ctx, C_MVP, c.mvp_idx);
    e.bin(ctx, C_RQT_ROOT, root_cbf);
    return root_cbf;
}

// One 16x16 transform node of unit c at depth d (0: a CU16's tree, 1: a quadrant of a CU32's),
// up to its children / residual: split_transform_flag (while d < depth = max_transform_hierarchy_
// depth_inter or _intra, by the CU's prediction), chroma cbf (coded at depth 0, else when the parent's
// is set; context = depth), and for an unsplit node cbf_luma (inferred 1 for an inter node at depth 0
// without chroma; context 1 at depth 0) and cu_qp_delta when a level is coded and the CU's delta is
// still pending.
template <class E, class Ctx>
MXHD void code_node16(E& e, Ctx& ctx, const CuInfo& c, int d, int pcb, int pcr, int depth, bool qp_pending,
                      int qp_pred) {
    const bool intra = c.type == kCuIntra;
    const int cb = (c.cbf >> 1) & 1, cr = (c.cbf >> 2) & 1, cy = c.cbf & 1;
    const bool split = c.tu_split == 2;
    if (d < depth) e.bin(ctx, C_SPLIT_TRANSFORM + 1, split);  // ctxInc 5 - log2(16)
    if (d == 0 || pcb) e.bin(ctx, C_CBF_CHROMA + d, cb);
    if (d == 0 || pcr) e.bin(ctx, C_CBF_CHROMA + d, cr);
    if (split) return;
    if (intra || d > 0 || cb || cr) e.bin(ctx, C_CBF_LUMA + (d == 0 ? 1 : 0), cy);
    if (c.cbf && qp_pending) code_qp_delta(e, ctx, qp_delta_wrap(c.qp, qp_pred));
}

// Split tree: the transform unit that carries cu_qp_delta -- the first one in decoding order with a
// coded luma level or coded chroma at its node (a 4x4 luma TU sees its 8x8 node's chroma, 7.3.8.10
// cbfDepthC): 4k + j for 4x4 TU j of node k, 16 + k for an unsplit 8x8 node k, -1 for none.
MXHD int split_qp_tu(const CuInfo& c) {
    for (int k = 0; k < 4; ++k) {
        const bool ck = ((c.cbf_c4 >> k) & 1) | ((c.cbf_c4 >> (4 + k)) & 1);
        if ((c.tu4 >> k) & 1) {
            for (int j = 0; j < 4; ++j)
                if (ck || ((c.cbf_y16 >> (4 * k + j)) & 1)) return 4 * k + j;
        } else if (ck || ((c.cbf_y4 >> k) & 1)) {
            return 16 + k;
        }
    }
    return -1;
}
// 8x8 child k (depth d + 1) of a split 16x16 node at depth d; its chroma TUs are 4x4 at this node:
// split_transform_flag (tu4: four 4x4 luma TUs) while d + 1 < depth (the CU's max_transform_
// hierarchy_depth), chroma cbf when the parent's is set, and for an unsplit child cbf_luma (context 0)
// and cu_qp_delta when pending and this is its TU.
template <class E, class Ctx>
MXHD void code_child8(E& e, Ctx& ctx, const CuInfo& c, int k, int d, int depth, bool qp_pending, int qp_pred) {
    const int cb = (c.cbf >> 1) & 1, cr = (c.cbf >> 2) & 1;
    const int yk = (c.cbf_y4 >> k) & 1, cbk = (c.cbf_c4 >> k) & 1, crk = (c.cbf_c4 >> (4 + k)) & 1;
    const int s4 = (c.tu4 >> k) & 1;
    if (d + 1 < depth) e.bin(ctx, C_SPLIT_TRANSFORM + 2, s4);  // ctxInc 5 - log2(8)
    if (cb) e.bin(ctx, C_CBF_CHROMA + d + 1, cbk);
    if (cr) e.bin(ctx, C_CBF_CHROMA + d + 1, crk);
    if (s4) return;  // the four 4x4 TUs code their own cbf_luma (code_grand4)
    e.bin(ctx, C_CBF_LUMA + 0, yk);
    if (qp_pending && split_qp_tu(c) == 16 + k) code_qp_delta(e, ctx, qp_delta_wrap(c.qp, qp_pred));
}
// 4x4 luma TU j of split child k (depth d + 2): cbf_luma (context 0), cu_qp_delta when pending
// and this is its TU
template <class E, class Ctx>
MXHD void code_grand4(E& e, Ctx& ctx, const CuInfo& c, int k, int j, bool qp_pending, int qp_pred) {
    e.bin(ctx, C_CBF_LUMA + 0, (c.cbf_y16 >> (4 * k + j)) & 1);
    if (qp_pending && split_qp_tu(c) == 4 * k + j) code_qp_delta(e, ctx, qp_delta_wrap(c.qp, qp_pred));
}
// Whether TU t (0 Y, 1 Cb, 2 Cr) of split child k is coded, and its first CU sub-block.
MXHD bool split_tu_coded(const CuInfo& c, int k, int t) {
    return t == 0 ? ((c.cbf_y4 >> k) & 1) : ((c.cbf_c4 >> (t == 1 ? k : 4 + k)) & 1);
}
MXHD int split_tu_sb0(int k, int t) { return t == 0 ? 4 * k : (t == 1 ? 16 + k : 20 + k); }
// scanIdx of the split tree's TUs of CU c (8x8 / 4x4 luma and 4x4 chroma; DM chroma)
MXHD int split_scan(const CuInfo& c) { return c.type == kCuIntra ? intra_scan_idx(c.intra_mode) : 0; }
// TU descriptor of a split child's TU / an unsplit unit's TU
template <class Cf>
MXHD TuDesc split_tu_desc(const Cf& cf, int k, int t, int scan) {
    TuDesc d;
    d.sb0 = split_tu_sb0(k, t);
    d.log2n = t == 0 ? 3 : 2;
    d.cidx = t;
    d.last_idx = tu_last(cf, d.sb0, t == 0 ? 4 : 1, &d.csbf_mask);
    d.scan = scan;
    return d;
}
// the 4x4 luma TU j of split child k (one sub-block: 4k + j)
template <class Cf>
MXHD TuDesc luma4_tu_desc(const Cf& cf, int k, int j, int scan) {
    TuDesc d;
    d.sb0 = 4 * k + j;
    d.log2n = 2;
    d.cidx = 0;
    d.last_idx = tu_last(cf, d.sb0, 1, &d.csbf_mask);
    d.scan = scan;
    return d;
}
MXHD TuDesc flat_tu_desc(const CuInfo& c, int t) {
    TuDesc d;
    d.scan = 0;
    d.sb0 = t == 0 ? 0 : (t == 1 ? 16 : 20);
    d.log2n = t == 0 ? 4 : 3;
    d.cidx = t;
    d.last_idx = t == 0 ? c.last[0] : (t == 1 ? c.last[1] : c.last[2]);
    d.csbf_mask = t == 0 ? c.csbf_y : (t == 1 ? c.csbf_c[0] : c.csbf_c[1]);
    return d;
}

// Everything the syntax of one unit needs beyond its own CuInfo and levels (unit_syn builds it).
struct UnitSyn {
    bool islice;
    bool ctb_first;    // z == 0: sao() and the CTB's split_cu_flag precede the unit
    bool split_coded;  // the CTB lies inside the picture (else split_cu_flag is inferred 1)
    int split_inc;     // split_cu_flag ctxInc at depth 0
    bool cu32;         // the CTB is one CU32
    bool root;         // a transform tree follows the CU's prediction syntax
    int cb0, cr0;      // CU32: depth-0 chroma cbf (OR over the units)
    bool qp_pending;   // the CU has not sent cu_qp_delta before this unit
    int qp_pred;       // qPY_PRED of the CU's quantization group (slice_qp_chain)
    CuNb nb;           // neighbours of the CU origin (a CU32: its first unit)
    CuInfo head;       // CU32: prediction info of the first unit with cbf = OR over the units
    bool last_unit;    // the CTB's last unit inside the picture: end_of_slice_segment_flag follows
    bool eos;          // ... equal to 1 (the slice's last CTB)
    bool end_subset;   // WPP: end_of_subset_one_bit (the last CTB of a CTB row, not of the slice)
    int depth_inter;   // max_transform_hierarchy_depth_inter
    int depth_intra;   // max_transform_hierarchy_depth_intra
    MXHD int depth_of(const CuInfo& c) const { return c.type == kCuIntra ? depth_intra : depth_inter; }
    bool sao_on, has_l, has_u;
    uint32_t sao[3], sao_l[3], sao_u[3];
};

// Build the syntax context of unit (x, y) of a slice of CTBs [first_ctb, end_ctb).  get(u): CuInfo
// of raster unit u; sao: 4 words per CTB (nullptr: SAO off); qp_pred: the unit's QP predictor.
template <class Get>
MXHD UnitSyn unit_syn(const Get& get, const uint32_t* sao, int x, int y, int mb_w, int mb_h, bool islice,
                      int first_ctb, int end_ctb, bool wpp, int depth_inter, int depth_intra, int qp_pred) {
    UnitSyn u;
    const int cw = ctb_cols(mb_w);
    const int c = ctb_of(x, y, cw), z = ((y & 1) << 1) | (x & 1);
    const int x0 = x & ~1, y0 = y & ~1;
    const CuInfo me = get(y * mb_w + x);
    u.islice = islice;
    u.ctb_first = z == 0;
    u.split_coded = ctb_whole(c, cw, mb_w, mb_h);
    u.cu32 = me.ct == 0;
    u.depth_inter = depth_inter;
    u.depth_intra = depth_intra;
    u.qp_pred = qp_pred;
    u.nb = cu_nb_at(get, u.cu32 ? x0 : x, u.cu32 ? y0 : y, mb_w, cw, first_ctb);
    u.split_inc = 0;
    if (x0 > 0 && c - 1 >= first_ctb) u.split_inc += get(y0 * mb_w + x0 - 1).ct > 0 ? 1 : 0;
    if (y0 > 0 && c - cw >= first_ctb) u.split_inc += get((y0 - 1) * mb_w + x0).ct > 0 ? 1 : 0;
    u.qp_pending = true;
    u.cb0 = u.cr0 = 0;
    if (u.cu32) {
        u.head = get(y0 * mb_w + x0);
        uint32_t any = 0;
        for (int q = 0; q < 4; ++q) {
            const uint32_t cb = get((y0 + (q >> 1)) * mb_w + x0 + (q & 1)).cbf;
            any |= cb;
            if (q < z && cb) u.qp_pending = false;
        }
        u.head.cbf = (uint8_t)any;
        u.cb0 = (int)((any >> 1) & 1);
        u.cr0 = (int)((any >> 2) & 1);
        u.root = u.head.type == kCuMerge || (u.head.type == kCuAmvp && any != 0) || u.head.type == kCuIntra;
    } else {
        u.head = me;
        u.root = me.type == kCuIntra || me.type == kCuMerge || (me.type == kCuAmvp && me.cbf != 0);
    }
    const int lz = ctb_last_z(c, cw, mb_w, mb_h);
    u.last_unit = z == lz;
    u.eos = c == end_ctb - 1;
    u.end_subset = wpp && !u.eos && (c % cw) == cw - 1;
    u.sao_on = sao != nullptr;
    u.has_l = (c % cw) > 0 && c - 1 >= first_ctb;
    u.has_u = c - cw >= first_ctb;
    for (int k = 0; k < 3; ++k) {
        u.sao[k] = sao ? sao[4 * (size_t)c + k] : 0u;
        u.sao_l[k] = (sao && u.has_l) ? sao[4 * (size_t)(c - 1) + k] : 0u;
        u.sao_u[k] = (sao && u.has_u) ? sao[4 * (size_t)(c - cw) + k] : 0u;
    }
    return u;
}

// How a unit's residual is laid out after its head part (code_unit_head): none, one transform
// unit per component, or the split tree (four 8x8 children, each with its own flags).
enum CuResidual { kResNone = 0, kResFlat = 1, kResSplit = 2 };
MXHD int unit_res_kind(const CuInfo& c, const UnitSyn& u) {
    if (!u.root) return kResNone;
    if (c.tu_split == 2) return kResSplit;
    return c.cbf ? kResFlat : kResNone;
}

// The unit's syntax before its split children / residual: [first unit of a CTB: sao() and
// split_cu_flag], then a CU32's prediction syntax and depth-0 chroma cbf (first unit) and the
// unit's depth-1 node, or a CU16's prediction syntax and depth-0 node.
template <class E, class Ctx>
MXHD void code_unit_head(E& e, Ctx& ctx, const CuInfo& c, const UnitSyn& u) {
    if (u.ctb_first) {
        if (u.sao_on)
            code_sao_w(e, ctx, u.sao[0], u.sao[1], u.sao[2], u.has_l, u.sao_l[0], u.sao_l[1], u.sao_l[2], u.has_u,
                       u.sao_u[0], u.sao_u[1], u.sao_u[2]);
        if (u.split_coded) e.bin(ctx, C_SPLIT_CU + u.split_inc, u.cu32 ? 0 : 1);
    }
    if (u.cu32) {
        if (u.ctb_first) {
            code_pred_head(e, ctx, u.islice, u.head, u.nb, u.head.cbf != 0, kCtbLog2);
            if (u.root) {
                e.bin(ctx, C_CBF_CHROMA + 0, u.cb0);
                e.bin(ctx, C_CBF_CHROMA + 0, u.cr0);
            }
        }
        if (u.root) code_node16(e, ctx, c, 1, u.cb0, u.cr0, u.depth_of(c), u.qp_pending, u.qp_pred);
        return;
    }
    // a CU16 (no split_cu_flag at depth 1 while the minimum CU is 16x16)
    if (code_pred_head(e, ctx, u.islice, c, u.nb, c.cbf != 0, kMinCbLog2))
        code_node16(e, ctx, c, 0, 0, 0, u.depth_of(c), true, u.qp_pred);
}
// split child k's head at the unit's tree depth, and the flags of its 4x4 TU j
template <class E, class Ctx>
MXHD void code_unit_child(E& e, Ctx& ctx, const CuInfo& c, const UnitSyn& u, int k) {
    code_child8(e, ctx, c, k, u.cu32 ? 1 : 0, u.depth_of(c), u.qp_pending, u.qp_pred);
}
template <class E, class Ctx>
MXHD void code_unit_grand(E& e, Ctx& ctx, const CuInfo& c, const UnitSyn& u, int k, int j) {
    code_grand4(e, ctx, c, k, j, u.qp_pending, u.qp_pred);
}
// end_of_slice_segment_flag after the CTB's last unit (+ end_of_subset_one_bit with WPP)
template <class E>
MXHD void code_unit_end(E& e, const UnitSyn& u) {
    if (!u.last_unit) return;
    e.terminate(u.eos ? 1 : 0);
    if (u.end_subset) e.terminate(1);
}

// ---------------------------------------------------------------- sample adaptive offset (8.7.3)
// Decided per CTB on the deblocked picture: for every component the rate-distortion best of
// off / band offset (four consecutive 8-wide bands) / edge offset (classes 0..3), with offsets
// from the rounded mean error of each category, shortened toward 0 while that lowers
// 16 * dSSE + lambda16 * bits (kLambdaSse16).  Cb and Cr share the type and edge class.  The
// choice depends on the CTB's own statistics only, and sao_merge_left / _up are sent exactly when
// the neighbour's parameters are identical -- so the decision is CTB-parallel on the GPU and
// merging never changes a CTB's parameters.
//
// One component's parameters in a word: bits 0-1 SaoTypeIdx (0 off, 1 band, 2 edge), 2-3 edge
// class, 4-8 sao_band_position, 12 + 4k .. 15 + 4k SaoOffsetVal[k + 1] (4-bit two's complement).
MXHD uint32_t sao_pack(int type, int eo, int band, const int* off) {
    uint32_t w = (uint32_t)type | ((uint32_t)eo << 2) | ((uint32_t)band << 4);
    for (int k = 0; k < 4; ++k) w |= ((uint32_t)off[k] & 15u) << (12 + 4 * k);
    return w;
}
MXHD int sao_type(uint32_t w) { return (int)(w & 3); }
MXHD int sao_eo(uint32_t w) { return (int)((w >> 2) & 3); }
MXHD int sao_band(uint32_t w) { return (int)((w >> 4) & 31); }
MXHD int sao_off(uint32_t w, int k) { return (int)(w << (16 - 4 * k)) >> 28; }

// edge classes (Table 8-13 hPos / vPos): neighbours a = (x + dx[0], y + dy[0]), b = (x + dx[1], ..)
constexpr int8_t kSaoDx[4][2] = {{-1, 1}, {0, 0}, {-1, 1}, {1, -1}};
constexpr int8_t kSaoDy[4][2] = {{0, 0}, {-1, 1}, {-1, 1}, {-1, 1}};
// edge category 0..4 of sample c between a and b (8.7.3.2: edgeIdx 0,1,2 -> 1,2,0)
MXHD int sao_edge_cat(int c, int a, int b) {
    const int e = 2 + ((c > a) - (c < a)) + ((c > b) - (c < b));
    return e == 2 ? 0 : (e < 2 ? e + 1 : e);
}

// One component of one CTB: sums of (source - deblocked) and sample counts per edge class and
// category (1..4 -> index 0..3), and per band (sample >> 3).
struct SaoStats {
    int32_t eo_sum[4][4];
    int32_t eo_cnt[4][4];
    int32_t bo_sum[32];
    int32_t bo_cnt[32];
};

// Statistics of the nw x nh block at (x0, y0) of a W x H plane: rec / src at (x, y) are
// p[y * pitch + x * step] (step 2: one component of interleaved chroma).  Samples whose
// neighbour lies outside the picture are not modified by an edge class (8.7.3.2) and are left
// out of its statistics.
MXHD void sao_stats_block(const uint8_t* rec, int rpitch, const uint8_t* src, int spitch, int step, int x0, int y0,
                          int nw, int nh, int W, int H, SaoStats& st) {
    for (int k = 0; k < 4; ++k)
        for (int c = 0; c < 4; ++c) st.eo_sum[k][c] = st.eo_cnt[k][c] = 0;
    for (int b = 0; b < 32; ++b) st.bo_sum[b] = st.bo_cnt[b] = 0;
    for (int y = y0; y < y0 + nh; ++y)
        for (int x = x0; x < x0 + nw; ++x) {
            const int c = rec[y * rpitch + x * step];
            const int d = (int)src[y * spitch + x * step] - c;
            st.bo_sum[c >> 3] += d;
            st.bo_cnt[c >> 3] += 1;
            for (int k = 0; k < 4; ++k) {
                const int ax = x + kSaoDx[k][0], ay = y + kSaoDy[k][0], bx = x + kSaoDx[k][1], by = y + kSaoDy[k][1];
                if (ax < 0 || ay < 0 || bx < 0 || by < 0 || ax >= W || bx >= W || ay >= H || by >= H) continue;
                const int cat = sao_edge_cat(c, rec[ay * rpitch + ax * step], rec[by * rpitch + bx * step]);
                if (cat) {
                    st.eo_sum[k][cat - 1] += d;
                    st.eo_cnt[k][cat - 1] += 1;
                }
            }
        }
}

MXHD int sao_offset_bits(int a) { return a < 7 ? a + 1 : 7; }  // sao_offset_abs: TR, cMax 7, bypass
// Best offset in [lo, hi] for a category / band with error sum s over n samples: start at the
// rounded mean, step toward 0, keep the lowest 16 * (n o^2 - 2 o s) + lambda16 * bits (o = 0:
// no distortion change, one bin).  Returns that cost.  All costs fit 32 bits: n <= 256,
// |s| <= 255 n, |o| <= 7 give |16 dSSE| < 15M per offset and < 36M for a whole CTB choice.
MXHD int sao_best_offset(int s, int n, int lo, int hi, bool sign_bit, uint32_t lam16, int* o_out) {
    int o = 0;
    if (n > 0) o = s >= 0 ? (s + n / 2) / n : -((-s + n / 2) / n);
    o = o < lo ? lo : (o > hi ? hi : o);
    int best = (int)lam16;
    int best_o = 0;
    for (int v = o; v != 0; v += v > 0 ? -1 : 1) {
        const int a = v < 0 ? -v : v;
        const int j = 16 * (n * v * v - 2 * v * s) + (int)lam16 * (sao_offset_bits(a) + (sign_bit ? 1 : 0));
        if (j < best) {
            best = j;
            best_o = v;
        }
    }
    *o_out = best_o;
    return best;
}

// Per-component candidates: each edge class with its four offsets, and the best band window.
struct SaoCompChoice {
    int j_eo[4];
    int j_bo;
    int eo_off[4][4];
    int bo_off[4];
    int band;
};
// Band window of four consecutive bands (wrapping) with the lowest summed cost; the first
// position wins ties.
MXHD void sao_eval_comp(const SaoStats& st, uint32_t lam16, SaoCompChoice& ch) {
    for (int k = 0; k < 4; ++k) {
        int j = 0;
        for (int c = 0; c < 4; ++c)  // categories 1, 2 (valleys) positive, 3, 4 (peaks) negative
            j += sao_best_offset(st.eo_sum[k][c], st.eo_cnt[k][c], c < 2 ? 0 : -7, c < 2 ? 7 : 0, false, lam16,
                                 &ch.eo_off[k][c]);
        ch.j_eo[k] = j;
    }
    int jb[32], ob[32];
    for (int b = 0; b < 32; ++b) jb[b] = sao_best_offset(st.bo_sum[b], st.bo_cnt[b], -7, 7, true, lam16, &ob[b]);
    ch.j_bo = 0;
    ch.band = 0;
    for (int p = 0; p < 32; ++p) {
        const int j = jb[p] + jb[(p + 1) & 31] + jb[(p + 2) & 31] + jb[(p + 3) & 31];
        if (p == 0 || j < ch.j_bo) {
            ch.j_bo = j;
            ch.band = p;
        }
    }
    for (int k = 0; k < 4; ++k) ch.bo_off[k] = ob[(ch.band + k) & 31];
}
// Final parameters of a CTB (w[0] luma, w[1] Cb, w[2] Cr) from the three components' candidates.
// Syntax bits beyond the offsets: type (1 context bin + 1 bypass), band position 5, edge class 2.
MXHD void sao_combine(const SaoCompChoice& y, const SaoCompChoice& cb, const SaoCompChoice& cr, uint32_t lam16,
                      uint32_t* w) {
    const int lam = (int)lam16;
    {
        int best = lam;  // off: one bin
        w[0] = 0;
        const int jb = y.j_bo + lam * 7;
        if (jb < best) {
            best = jb;
            w[0] = sao_pack(1, 0, y.band, y.bo_off);
        }
        for (int k = 0; k < 4; ++k) {
            const int je = y.j_eo[k] + lam * 4;
            if (je < best) {
                best = je;
                w[0] = sao_pack(2, k, 0, y.eo_off[k]);
            }
        }
    }
    int best = lam;
    w[1] = w[2] = 0;
    const int jb = cb.j_bo + cr.j_bo + lam * 12;
    if (jb < best) {
        best = jb;
        w[1] = sao_pack(1, 0, cb.band, cb.bo_off);
        w[2] = sao_pack(1, 0, cr.band, cr.bo_off);
    }
    for (int k = 0; k < 4; ++k) {
        const int je = cb.j_eo[k] + cr.j_eo[k] + lam * 4;
        if (je < best) {
            best = je;
            w[1] = sao_pack(2, k, 0, cb.eo_off[k]);
            w[2] = sao_pack(2, k, 0, cr.eo_off[k]);
        }
    }
}

// SAO output of sample c (deblocked) with parameters w; a / b: its class-eo neighbours, or -1
// when one lies outside the picture (edge offset: unmodified).
// SAO output of sample c with parameters w when its edge category (class sao_eo(w)) is cat
// (0: flat, or a neighbour outside the picture).
MXHD int sao_sample_cat(uint32_t w, int c, int cat) {
    const int type = sao_type(w);
    int o = 0;
    if (type == 1) {
        const int k = ((c >> 3) - sao_band(w)) & 31;
        o = k < 4 ? sao_off(w, k) : 0;
    } else if (type == 2) {
        o = cat ? sao_off(w, cat - 1) : 0;
    }
    const int v = c + o;
    return v < 0 ? 0 : (v > 255 ? 255 : v);
}
MXHD int sao_sample(uint32_t w, int c, int a, int b) {
    return sao_sample_cat(w, c, (a >= 0 && b >= 0) ? sao_edge_cat(c, a, b) : 0);
}
// Encoder decision shared by both encoders: a CTB of a P picture whose CU coded no residual keeps
// its samples (SAO off) without gathering statistics.  Its prediction came from a picture SAO
// already corrected (static or rigidly moving content: most of a desktop), so a second offset pass
// finds ~nothing, and the statistics pass is the bulk of k_hevc_sao's time.
// (A CTB of several units keeps its samples when none of them coded a level.)
MXHD bool sao_keep_ctb(bool idr, uint32_t cbf_any) { return !idr && cbf_any == 0; }

// Apply w to the nw x nh block at (x0, y0): reads the deblocked plane rec, writes out (a different
// buffer: every CTB reads its neighbours' deblocked samples).
MXHD void sao_apply_block(const uint8_t* rec, uint8_t* out, int pitch, int step, int x0, int y0, int nw, int nh, int W,
                          int H, uint32_t w) {
    const int k = sao_eo(w);
    for (int y = y0; y < y0 + nh; ++y)
        for (int x = x0; x < x0 + nw; ++x) {
            const int ax = x + kSaoDx[k][0], ay = y + kSaoDy[k][0], bx = x + kSaoDx[k][1], by = y + kSaoDy[k][1];
            const bool in = ax >= 0 && ay >= 0 && bx >= 0 && by >= 0 && ax < W && bx < W && ay < H && by < H;
            const int a = in ? rec[ay * pitch + ax * step] : -1, b = in ? rec[by * pitch + bx * step] : -1;
            out[y * pitch + x * step] = (uint8_t)sao_sample(w, rec[y * pitch + x * step], a, b);
        }
}

// sao(rx, ry) syntax (7.3.8.3) of a CTB with parameters (p0, p1, p2); the left / up neighbour
// CTB's parameters count only when it is in the slice (has_l / has_u).  Values, not pointers:
// on the device every argument stays in (wave-uniform) registers.
template <class E, class Ctx>
MXHD void code_sao_w(E& e, Ctx& ctx, uint32_t p0, uint32_t p1, uint32_t p2, bool has_l, uint32_t l0,
                     uint32_t l1, uint32_t l2, bool has_u, uint32_t u0, uint32_t u1, uint32_t u2) {
    if (has_l) {
        const bool m = l0 == p0 && l1 == p1 && l2 == p2;
        e.bin(ctx, C_SAO_MERGE, m ? 1 : 0);
        if (m) return;
    }
    if (has_u) {
        const bool m = u0 == p0 && u1 == p1 && u2 == p2;
        e.bin(ctx, C_SAO_MERGE, m ? 1 : 0);
        if (m) return;
    }
    for (int c = 0; c < 3; ++c) {
        const uint32_t w = c == 0 ? p0 : (c == 1 ? p1 : p2);
        const int type = sao_type(w);
        if (c < 2) {
            e.bin(ctx, C_SAO_TYPE, type != 0 ? 1 : 0);
            if (type) e.bypass(type == 2 ? 1 : 0);
        }
        if (!type) continue;
        for (int k = 0; k < 4; ++k) {
            const int o = sao_off(w, k), a = o < 0 ? -o : o;
            if (a < 7)
                e.bypass_bits(((1u << a) - 1u) << 1, a + 1);  // a ones, then a zero
            else
                e.bypass_bits(0x7fu, 7);
        }
        if (type == 1) {
            for (int k = 0; k < 4; ++k)
                if (sao_off(w, k)) e.bypass(sao_off(w, k) < 0 ? 1 : 0);
            e.bypass_bits((uint32_t)sao_band(w), 5);
        } else if (c < 2) {
            e.bypass_bits((uint32_t)sao_eo(w), 2);
        }
    }
}
template <class E, class Ctx>
MXHD void code_sao(E& e, Ctx& ctx, const uint32_t* p, const uint32_t* left, const uint32_t* up) {
    code_sao_w(e, ctx, p[0], p[1], p[2], left != nullptr, left ? left[0] : 0u, left ? left[1] : 0u,
               left ? left[2] : 0u, up != nullptr, up ? up[0] : 0u, up ? up[1] : 0u, up ? up[2] : 0u);
}

// ---------------------------------------------------------------- bin tokens
// Entropy coding in two phases: a CTU's syntax is first *binarised* into 16-bit tokens (which
// bins, with which context -- a pure function of the CTU, its neighbours' descriptors and the
// QP predictor, so every CTU of a picture can be binarised in parallel), then a slice's token
// stream runs through the arithmetic coder, the only serial part (a short loop per token with
// no syntax logic).  Token layout:
//   bit 15 = 0: context-coded bin, bits 1..8 context index (kTokTerm: end_of_slice terminate
//               bin), bit 0 the bin value;
//   bit 15 = 1: a run of n = bits 11..14 + 1 (<= 11) bypass bins, value bits 0..10 (MSB first).
constexpr uint32_t kTokTerm = 255;
constexpr int kTokBypassMax = 11;
// Upper bound of the tokens of one CTU: 24 coded sub-blocks of at most 1 csbf + 16 sig + 8 gt1 +
// 1 gt2 + 2 sign + 16 * 5 remaining (escape prefix, EGk prefix and suffix split at 11 bins), plus
// the last-position, CU and SAO syntax.
constexpr uint32_t kMaxCuTokens = 24 * 108 + 256;

// Records bins as tokens (same interface as CabacEnc).  Consecutive bypass bins are merged.
struct BinRec {
    uint16_t* out;
    uint32_t n, cap;
    uint32_t pv;
    int pn;
    MXHD void start(uint16_t* o, uint32_t c) {
        out = o;
        n = 0;
        cap = c;
        pv = 0;
        pn = 0;
    }
    MXHD void put(uint32_t t) {
        if (n < cap) out[n] = (uint16_t)t;
        ++n;
    }
    MXHD void flush() {
        if (pn) put(0x8000u | ((uint32_t)(pn - 1) << 11) | pv);
        pv = 0;
        pn = 0;
    }
    template <class Ctx>
    MXHD void bin(Ctx&, int idx, int b) {
        flush();
        put(((uint32_t)idx << 1) | (uint32_t)b);
    }
    MXHD void terminate(int b) {
        flush();
        put((kTokTerm << 1) | (uint32_t)b);
    }
    MXHD void bypass_bits(uint32_t v, int n) {
        while (n > 0) {
            const int k = n < kTokBypassMax - pn ? n : kTokBypassMax - pn;
            n -= k;
            pv = (pv << k) | ((v >> n) & ((1u << k) - 1u));
            pn += k;
            if (pn == kTokBypassMax) flush();
        }
    }
    MXHD void bypass(int b) { bypass_bits((uint32_t)b, 1); }
};
struct NoCtx {};

// Token -> arithmetic coder.
template <class Ctx>
MXHD void code_token(CabacEnc& e, Ctx& ctx, uint32_t t) {
    if (t & 0x8000u)
        e.bypass_bits(t & 0x7ffu, (int)((t >> 11) & 15u) + 1);
    else if ((t >> 1) == kTokTerm)
        e.terminate((int)(t & 1u));
    else
        e.bin(ctx, (int)(t >> 1), (int)(t & 1u));
}

// A unit's token stream is the concatenation of independent *parts* in coding order: the head
// (code_unit_head: sao() and split_cu_flag on a CTB's first unit, the prediction syntax, the
// 16x16 transform node), per split child its flags / cu_qp_delta, per TU its last position and
// its sub-blocks (last to DC), and on the CTB's last unit the end_of_slice_segment_flag.  Each part
// depends only on the unit, its neighbours' descriptors and UnitSyn, so the GPU binarises one
// part per lane (k_hevc_bins); the CPU walks them in order.  At most 1 + 4 + 12 + 24 + 1 = 42
// parts; a part is at most kPartTokens tokens.
// A split child whose luma is four 4x4 TUs has one part per 4x4 TU (kPartGrand: its cbf_luma,
// cu_qp_delta and, when coded, its last position) followed by the TU's one sub-block, then its
// chroma TUs.  Worst case 1 + 4 + 16 x 2 + 8 x 2 + 1 = 54 parts (one wave).
enum PartKind { kPartHead = 0, kPartChild = 1, kPartTuLast = 2, kPartSb = 3, kPartEnd = 4, kPartGrand = 5 };
struct CtuPart {
    int kind, k, t, i;  // split child, component TU (or 4x4 luma TU j of kPartGrand), sub-block index within the TU
    TuDesc d;           // TU of kPartTuLast / kPartSb / a coded kPartGrand
};
constexpr int kMaxCtuParts = 54;
constexpr uint32_t kPartTokens = 112;

// Calls f(part, index) for every part of unit c in coding order; returns the number of parts.
template <class Cf, class F>
MXHD int for_each_part(const CuInfo& c, const UnitSyn& u, const Cf& cf, F f) {
    int n = 0;
    CtuPart pt;
    pt.kind = kPartHead;
    pt.k = pt.t = pt.i = 0;
    f(pt, n++);
    const int kind = unit_res_kind(c, u);
#pragma unroll 1
    for (int k = 0; k < (kind == kResSplit ? 4 : 1); ++k) {
        if (kind == kResNone) break;
        if (kind == kResSplit) {
            pt.kind = kPartChild;
            pt.k = k;
            f(pt, n++);
        }
        const bool s4 = kind == kResSplit && ((c.tu4 >> k) & 1);
        if (s4) {
#pragma unroll 1
            for (int j = 0; j < 4; ++j) {
                const bool coded = (c.cbf_y16 >> (4 * k + j)) & 1;
                if (coded) pt.d = luma4_tu_desc(cf, k, j, split_scan(c));
                pt.k = k;
                pt.t = j;
                pt.kind = kPartGrand;
                f(pt, n++);
                if (coded) {
                    pt.kind = kPartSb;
                    pt.i = 0;
                    f(pt, n++);
                }
            }
        }
#pragma unroll 1
        for (int t = s4 ? 1 : 0; t < 3; ++t) {
            const bool coded = kind == kResSplit ? split_tu_coded(c, k, t) : (((c.cbf >> t) & 1) != 0);
            if (!coded) continue;
            pt.d = kind == kResSplit ? split_tu_desc(cf, k, t, split_scan(c)) : flat_tu_desc(c, t);
            pt.k = k;
            pt.t = t;
            pt.kind = kPartTuLast;
            f(pt, n++);
            pt.kind = kPartSb;
#pragma unroll 1
            for (int i = pt.d.last_idx >> 4; i >= 0; --i) {
                pt.i = i;
                f(pt, n++);
            }
        }
    }
    if (u.last_unit) {
        pt.kind = kPartEnd;
        f(pt, n++);
    }
    return n;
}

// Binarise one part of unit c (E: BinRec with NoCtx, or the arithmetic coder with ArrCtx).
template <class E, class Ctx, class Cf>
MXHD void binarise_part(E& rec, Ctx& ctx, const CtuPart& pt, const CuInfo& c, const UnitSyn& u, const Cf& cf) {
    if (pt.kind == kPartHead) {
        code_unit_head(rec, ctx, c, u);
    } else if (pt.kind == kPartChild) {
        code_unit_child(rec, ctx, c, u, pt.k);
    } else if (pt.kind == kPartGrand) {
        code_unit_grand(rec, ctx, c, u, pt.k, pt.t);
        if ((c.cbf_y16 >> (4 * pt.k + pt.t)) & 1) code_tu_last(rec, ctx, pt.d);
    } else if (pt.kind == kPartTuLast) {
        code_tu_last(rec, ctx, pt.d);
    } else if (pt.kind == kPartSb) {
        // the previous sub-block with levels in this TU (coding order: higher scan index)
        const int last_sb = pt.d.last_idx >> 4;
        int prev_gt1 = -1;
        for (int j = pt.i + 1; j <= last_sb; ++j) {
            if (!(j == last_sb || ((pt.d.csbf_mask >> j) & 1))) continue;
            const uint32_t sg = cf.sig(pt.d.sb0 + j);
            if (!sg) continue;
            prev_gt1 = sb_any_gt1(cf, pt.d.sb0 + j, sg) ? 1 : 0;
            break;
        }
        code_sub_block(rec, ctx, cf, pt.d, tu_csbf_raster(pt.d), pt.i, prev_gt1);
    } else {
        code_unit_end(rec, u);
    }
    rec.flush();
}

// A unit coded straight through the syntax coders (the residual coder walks each TU in one
// pass): the reference the part-wise token path is tested against.
template <class E, class Ctx, class Cf>
MXHD void code_unit_direct(E& e, Ctx& ctx, const CuInfo& c, const UnitSyn& u, const Cf& cf) {
    code_unit_head(e, ctx, c, u);
    const int kind = unit_res_kind(c, u);
    if (kind == kResSplit) {
#pragma unroll 1
        for (int k = 0; k < 4; ++k) {
            code_unit_child(e, ctx, c, u, k);
            const bool s4 = (c.tu4 >> k) & 1;
            if (s4)
                for (int j = 0; j < 4; ++j) {
                    code_unit_grand(e, ctx, c, u, k, j);
                    if ((c.cbf_y16 >> (4 * k + j)) & 1) code_residual(e, ctx, cf, luma4_tu_desc(cf, k, j, split_scan(c)));
                }
#pragma unroll 1
            for (int t = s4 ? 1 : 0; t < 3; ++t)
                if (split_tu_coded(c, k, t)) code_residual(e, ctx, cf, split_tu_desc(cf, k, t, split_scan(c)));
        }
    } else if (kind == kResFlat) {
#pragma unroll 1
        for (int t = 0; t < 3; ++t)
            if ((c.cbf >> t) & 1) code_residual(e, ctx, cf, flat_tu_desc(c, t));
    }
    code_unit_end(e, u);
}

// What the entropy coder reads of a picture: raster CuInfo / levels per unit, the QP predictor per
// unit (slice_qp_chain), SAO words per CTB (nullptr: off).
struct PicSyn {
    const CuInfo* cus;
    const int16_t* coef;
    const uint8_t* qp_pred;
    const uint32_t* sao;
    int mb_w, mb_h;
    int depth_inter;  // max_transform_hierarchy_depth_inter
    int depth_intra;  // max_transform_hierarchy_depth_intra
};
struct ArrGet {  // raster CuInfo lookup for unit_syn
    const CuInfo* p;
    MXHD const CuInfo& operator()(int u) const { return p[u]; }
};
MXHD UnitSyn pic_unit_syn(const PicSyn& ps, int x, int y, bool islice, int first, int end, bool wpp) {
    return unit_syn(ArrGet{ps.cus}, ps.sao, x, y, ps.mb_w, ps.mb_h, islice, first, end, wpp, ps.depth_inter,
                    ps.depth_intra, ps.qp_pred[y * ps.mb_w + x]);
}

// Entropy-code CTB c of the slice [first, end) into e: every unit inside the picture, in z order,
// through the token path (binarise, then the tokens through the coder -- what the GPU does) or
// directly (direct = true).
MXHD void code_ctb(CabacEnc& e, ArrCtx& ctx, const PicSyn& ps, bool islice, int c, int first, int end, bool wpp,
                   uint16_t* tok, bool direct) {
    const int cw = ctb_cols(ps.mb_w);
    for (int z = 0; z < 4; ++z) {
        const int x = 2 * (c % cw) + (z & 1), y = 2 * (c / cw) + (z >> 1);
        if (x >= ps.mb_w || y >= ps.mb_h) continue;
        const int i = y * ps.mb_w + x;
        const UnitSyn u = pic_unit_syn(ps, x, y, islice, first, end, wpp);
        const CoefArray cf{ps.coef + (size_t)i * kCoefPerCu};
        if (direct) {
            code_unit_direct(e, ctx, ps.cus[i], u, cf);
            continue;
        }
        BinRec rec;
        rec.start(tok, kMaxCuTokens);
        NoCtx nc;
        for_each_part(ps.cus[i], u, cf, [&](const CtuPart& pt, int) { binarise_part(rec, nc, pt, ps.cus[i], u, cf); });
        for (uint32_t j = 0; j < rec.n && j < kMaxCuTokens; ++j) code_token(e, ctx, tok[j]);
    }
}

// Entropy-code the slice of CTBs [first, end) (one substream).  Returns the payload bytes.
MXHD uint32_t code_slice(uint8_t* out, uint32_t cap, bool islice, int slice_qp, const PicSyn& ps, int first, int end,
                         uint8_t* ctx_mem, uint16_t* tok, bool direct = false) {
    ctx_init_all(ctx_mem, islice ? 0 : 1, slice_qp);
    ArrCtx ctx{ctx_mem};
    CabacEnc e;
    e.start(out, cap);
    for (int c = first; c < end; ++c) code_ctb(e, ctx, ps, islice, c, first, end, false, tok, direct);
    e.finish_slice();
    return e.pos;
}

// ---------------------------------------------------------------- encoder decisions
// Approximate luma mode signalling cost in bins given the MPM candidates of the left / above PU.
MXHD int intra_mode_bits(int mode, int cand_a, int cand_b) {
    int l[3];
    mpm_list(cand_a, cand_b, l);
    if (mode == l[0]) return 2;
    if (mode == l[1] || mode == l[2]) return 3;
    return 6;
}

// Coarse-to-fine order of the open-loop intra mode search (intra_decide_mode, k_hevc_intra_modes):
// planar, DC and every fourth angular mode, then the modes two and one away from the best angular
// mode so far -- at most 15 of the 35 predictions.  cost(m): the mode's cost, kIntraNoMode when the
// mode may not be used; the lowest cost wins, ties to the lower mode.
// Intra transform-tree split of a 16x16 unit (EncoderConfig::hevc_intra_split): four 8x8 luma TUs
// and per chroma component four 4x4 TUs, in z order, each predicted in the unit's mode (DM chroma)
// from the reconstruction of the TUs before it.  split_tu_avl: reference availability of TU k (bit 0
// below-left, 1 left, 2 corner, 3 top, 4 top-right -- the segments of intra_refs / ref_subst) from
// the unit's left / corner / top / top-right.  Inside the unit every decoded neighbour is there; not
// decoded yet: the below-left of TUs 1 and 3 and the top-right of TU 3.  TU 2's below-left is the
// unit below-left, which the decoder has only in a CTB's first unit (bl_pending) and the raster
// wavefront has not reconstructed then: such a unit splits only in a mode that never reads it
// (bl_safe_split) and predicts as if it were absent, as the unsplit unit does with bl_safe_modes.
MXHD int split_tu_avl(int k, bool al, bool ac, bool at, bool atr) {
    if (k == 0) return (al ? 3 : 0) | (ac ? 4 : 0) | (at ? 24 : 0);
    if (k == 1) return 2 | (at ? 12 : 0) | (atr ? 16 : 0);
    if (k == 2) return (al ? 6 : 0) | 24;
    return 14;
}
// modes whose 8x8 luma and 4x4 DM chroma predictions never read the below-left references
inline uint64_t bl_safe_split() { return bl_safe_modes(3, 0) & bl_safe_modes(2, 1); }
// Open-loop choice (from the source, luma only): split when the best split mode's cost (four TUs'
// 4x4 Hadamard SATD + lambda * mode bits) plus lambda * kIntraSplitBits (the split tree's extra cbf
// flags) is below the best unsplit mode's.  The imode byte carries it in bit 6.
constexpr int kIntraSplitBits = 10;
constexpr int kIntraSplitFlag = 64;
MXHD bool intra_split_wins(int cost16, int cost8, int lambda) { return cost8 + lambda * kIntraSplitBits < cost16; }
// a split cost is at least lambda * 2 (the cheapest mode signalling): below this unsplit cost the split
// search cannot win and is skipped (flat content; the decision is unchanged)
MXHD bool intra_split_possible(int cost16, int lambda) { return cost16 > lambda * (kIntraSplitBits + 2); }

constexpr int kIntraCoarse[11] = {0, 1, 2, 6, 10, 14, 18, 22, 26, 30, 34};
constexpr int kIntraNoMode = 0x7fffffff;
template <class F>
MXHD int intra_mode_search(const F& cost) {
    int best = 1, bc = kIntraNoMode, ba = -1, bac = kIntraNoMode;
    auto visit = [&](int m) {
        const int c = cost(m);
        if (c == kIntraNoMode) return;
        if (c < bc || (c == bc && m < best)) {
            bc = c;
            best = m;
        }
        if (m >= 2 && (c < bac || (c == bac && m < ba))) {
            bac = c;
            ba = m;
        }
    };
    for (int i = 0; i < 11; ++i) visit(kIntraCoarse[i]);
    if (ba >= 2) {
        const int a = ba;
        if (a - 2 >= 2) visit(a - 2);
        if (a + 2 <= 34) visit(a + 2);
        const int b = ba;
        if (b - 1 >= 2) visit(b - 1);
        if (b + 1 <= 34) visit(b + 1);
    }
    return best;
}

// Residual (raster NxN) -> quantised levels in scan order + reconstructed residual (raster).
// Returns the number of nonzero levels.
// Inter TU decimation: a TU whose only levels are a few +-1s is zeroed (it costs many
// significance bins and bits for a fraction of a dB; HM/x264 drop such blocks by RD or
// decimation scores).  Same rule in the CPU and GPU encoders.
// Trailing-level trim (inter): the last significant level is dropped while it is +-1 and
// more than kTrimGap zero positions separate it from the previous one (each costs a
// significance bin), at most kTrimIters times per TU.
constexpr int kTrimGap = 8;
constexpr int kTrimIters = 4;

MXHD bool tu_decimate(int log2n, bool intra, int nz, int max_abs) {
    return !intra && nz > 0 && max_abs == 1 && nz <= (log2n == 4 ? 4 : 2);
}

// Fixed-size forward / inverse transforms (same arithmetic as fwd_transform / inv_transform,
// arrays sized for the TU so per-lane GPU callers keep them out of scratch).
template <int L>
MXHD void fwd_transform_t(const int* res, int* out) {
    constexpr int N = 1 << L, s1 = L - 1, s2 = L + 6;
    int tmp[N * N];
    for (int y = 0; y < N; ++y)
        for (int k = 0; k < N; ++k) {
            int s = 0;
            for (int n = 0; n < N; ++n) s += dct_coef(L, k, n) * res[y * N + n];
            tmp[y * N + k] = (s + (1 << (s1 - 1))) >> s1;
        }
    for (int k2 = 0; k2 < N; ++k2)
        for (int k = 0; k < N; ++k) {
            int s = 0;
            for (int y = 0; y < N; ++y) s += dct_coef(L, k2, y) * tmp[y * N + k];
            out[k2 * N + k] = (s + (1 << (s2 - 1))) >> s2;
        }
}
template <int L>
MXHD void inv_transform_t(const int* d, int* r) {
    constexpr int N = 1 << L;
    int g[N * N];
    for (int x = 0; x < N; ++x)
        for (int y = 0; y < N; ++y) {
            int s = 0;
            for (int k = 0; k < N; ++k) s += dct_coef(L, k, y) * d[k * N + x];
            g[y * N + x] = clip16((s + 64) >> 7);
        }
    for (int y = 0; y < N; ++y)
        for (int x = 0; x < N; ++x) {
            int s = 0;
            for (int k = 0; k < N; ++k) s += dct_coef(L, k, x) * g[y * N + k];
            r[y * N + x] = (s + 2048) >> 12;
        }
}

template <int L>
MXHD int tu_encode_t(const int* res, int qp, bool intra, int16_t* levels, int* rres, int scan = 0) {
    constexpr int N = 1 << L;
    const int log2n = L;
    int c[N * N], d[N * N];
    fwd_transform_t<L>(res, c);
    int nz = 0, mx = 0;
    for (int v = 0; v < N; ++v)
        for (int u = 0; u < N; ++u) {
            const int l = quant_coef(c[v * N + u], qp, log2n, intra);
            c[v * N + u] = l;
            nz += l != 0;
            mx = (l < 0 ? -l : l) > mx ? (l < 0 ? -l : l) : mx;
        }
    const bool drop = tu_decimate(log2n, intra, nz, mx);
    for (int v = 0; v < N; ++v)
        for (int u = 0; u < N; ++u) levels[scan_index_s(log2n, scan, u, v)] = (int16_t)(drop ? 0 : c[v * N + u]);
    if (!intra) {  // trailing isolated +-1 levels (same rule as the GPU kernel)
        for (int it = 0; it < kTrimIters; ++it) {
            int last = -1, prev = -1;
            for (int i = 0; i < N * N; ++i)
                if (levels[i]) {
                    prev = last;
                    last = i;
                }
            if (last < 0 || (levels[last] != 1 && levels[last] != -1) || last - prev <= kTrimGap) break;
            levels[last] = 0;
        }
    }
    nz = 0;
    for (int v = 0; v < N; ++v)
        for (int u = 0; u < N; ++u) {
            const int l = levels[scan_index_s(log2n, scan, u, v)];
            nz += l != 0;
            d[v * N + u] = dequant_coef(l, qp, log2n);
        }
    if (nz)
        inv_transform_t<L>(d, rres);
    else
        for (int i = 0; i < N * N; ++i) rres[i] = 0;
    return nz;
}

MXHD int tu_encode(int log2n, const int* res, int qp, bool intra, int16_t* levels, int* rres, int scan = 0) {
    if (log2n == 2) return tu_encode_t<2>(res, qp, intra, levels, rres, scan);
    if (log2n == 3) return tu_encode_t<3>(res, qp, intra, levels, rres, scan);
    return tu_encode_t<4>(res, qp, intra, levels, rres);
}

// lambda for SSE decisions, HM's 0.57 * 2^((QP-12)/3), in 1/16 units (integer: CPU == GPU)
constexpr uint32_t kLambdaSse16[52] = {1,    1,    1,    1,    1,    2,     2,     3,     4,     5,     6,
                                       7,    9,    11,   14,   18,   23,    29,    36,    46,    58,    73,
                                       92,   116,  146,  184,  232,  292,   368,   463,   584,   735,   927,
                                       1167, 1471, 1853, 2335, 2942, 3706,  4669,  5883,  7412,  9339,  11766,
                                       14825, 18678, 23533, 29649, 37356, 47065, 59298, 74711};
// Rough CABAC bits of one TU's levels: ~3.5 bins per significant level plus the magnitude
// (Golomb-Rice growth), ~4 bits of last position / cbf overhead per coded TU.
MXHD uint32_t tu_bits_est(const int16_t* lv, int n) {
    uint32_t b = 0;
    bool any = false;
    for (int k = 0; k < n; ++k) {
        const int a = lv[k] < 0 ? -lv[k] : lv[k];
        if (!a) continue;
        any = true;
        b += 4 + 2 * (31 - __builtin_clz((uint32_t)a));
    }
    return any ? b + 4 : 1;
}
// Split wins when its SSE + lambda * bits is lower (costs in 1/16 units).
// The split tree is tried only for CUs whose unsplit tree coded at least one level: a residual
// that quantises to nothing in 16x16 / 8x8 TUs is (nearly always) coding noise of a static or
// well-predicted block, and skipping the second tree there halves the transform work of a desktop
// P picture.  Shared by both encoders.
MXHD bool split_worth_trying(int levels_unsplit) { return levels_unsplit > 0; }
MXHD int tu_levels(const int16_t* lv, int n) {
    int k = 0;
    for (int i = 0; i < n; ++i) k += lv[i] != 0;
    return k;
}
MXHD bool choose_split(uint64_t sse16, uint32_t bits16, uint64_t sse8, uint32_t bits8, int qp) {
    const uint64_t l = kLambdaSse16[qp < 0 ? 0 : (qp > 51 ? 51 : qp)];
    return sse8 * 16 + l * bits8 < sse16 * 16 + l * bits16;
}

// The split transform tree of an inter CU: luma node k is the 8x8 block (k & 1, k >> 1) of the
// 16x16 residual, chroma TU k the 4x4 block (k & 1, k >> 1) of each 8x8 chroma residual; levels
// go to the CU's sub-blocks 4k.. (luma), 16 + k (Cb), 20 + k (Cr), i.e. co + 64k,
// co + 256 + 16k, co + 320 + 16k, each TU in scan order.  rr / rrc: reconstructed residuals.
// With try4 a luma node is also coded as four 4x4 TUs (sub-block 4k + j = the 4x4 block (j & 1,
// j >> 1) of the node) and keeps them when their luma SSE + lambda * bits is lower (choose_split,
// the node's own distortion against pred + res); returns the mask of such nodes (CuInfo::tu4).
MXHD int split_encode(const int* res, const int (*rc)[64], int qp, int qpc, int16_t* co, int* rr, int (*rrc)[64],
                      const int* pred = nullptr, bool try4 = false) {
    int blk[64], rb[64];
    int tu4 = 0;
    for (int k = 0; k < 4; ++k) {
        const int bx = (k & 1) * 8, by = (k >> 1) * 8;
        for (int r = 0; r < 8; ++r)
            for (int q = 0; q < 8; ++q) blk[r * 8 + q] = res[(by + r) * 16 + bx + q];
        tu_encode(3, blk, qp, false, co + 64 * k, rb);
        for (int r = 0; r < 8; ++r)
            for (int q = 0; q < 8; ++q) rr[(by + r) * 16 + bx + q] = rb[r * 8 + q];
        if (!try4 || !split_worth_trying(tu_levels(co + 64 * k, 64))) continue;
        int16_t l4[64];
        int r4[64], b4[16], rb4[16];
        for (int j = 0; j < 4; ++j) {
            const int jx = (j & 1) * 4, jy = (j >> 1) * 4;
            for (int r = 0; r < 4; ++r)
                for (int q = 0; q < 4; ++q) b4[r * 4 + q] = blk[(jy + r) * 8 + jx + q];
            tu_encode(2, b4, qp, false, l4 + 16 * j, rb4);
            for (int r = 0; r < 4; ++r)
                for (int q = 0; q < 4; ++q) r4[(jy + r) * 8 + jx + q] = rb4[r * 4 + q];
        }
        uint64_t s8 = 0, s4 = 0;
        for (int r = 0; r < 8; ++r)
            for (int q = 0; q < 8; ++q) {
                const int o = (by + r) * 16 + bx + q, src = pred[o] + res[o];
                const int e8 = src - clip255(pred[o] + rb[r * 8 + q]), e4 = src - clip255(pred[o] + r4[r * 8 + q]);
                s8 += (uint64_t)(e8 * e8);
                s4 += (uint64_t)(e4 * e4);
            }
        uint32_t b4bits = 0;
        for (int j = 0; j < 4; ++j) b4bits += tu_bits_est(l4 + 16 * j, 16);
        if (choose_split(s8, tu_bits_est(co + 64 * k, 64), s4, b4bits, qp)) {
            tu4 |= 1 << k;
            for (int i = 0; i < 64; ++i) co[64 * k + i] = l4[i];
            for (int r = 0; r < 8; ++r)
                for (int q = 0; q < 8; ++q) rr[(by + r) * 16 + bx + q] = r4[r * 8 + q];
        }
    }
    for (int comp = 0; comp < 2; ++comp)
        for (int k = 0; k < 4; ++k) {
            const int bx = (k & 1) * 4, by = (k >> 1) * 4;
            for (int r = 0; r < 4; ++r)
                for (int q = 0; q < 4; ++q) blk[r * 4 + q] = rc[comp][(by + r) * 8 + bx + q];
            tu_encode(2, blk, qpc, false, co + 256 + 64 * comp + 16 * k, rb);
            for (int r = 0; r < 4; ++r)
                for (int q = 0; q < 4; ++q) rrc[comp][(by + r) * 8 + bx + q] = rb[r * 4 + q];
        }
    return tu4;
}

// Estimated level bits of a CU's transform tree (unsplit: 16x16 + 2 x 8x8; split: per luma node
// one 8x8 or (tu4) four 4x4, + 8 x 4x4 chroma).
MXHD uint32_t cu_bits_est(const int16_t* co, bool split, int tu4 = 0) {
    if (!split) return tu_bits_est(co, 256) + tu_bits_est(co + 256, 64) + tu_bits_est(co + 320, 64);
    uint32_t b = 0;
    for (int k = 0; k < 4; ++k) {
        if ((tu4 >> k) & 1)
            for (int j = 0; j < 4; ++j) b += tu_bits_est(co + 64 * k + 16 * j, 16);
        else
            b += tu_bits_est(co + 64 * k, 64);
    }
    for (int k = 0; k < 8; ++k) b += tu_bits_est(co + 256 + 16 * k, 16);
    return b;
}

// Estimated bits of the luma levels alone (the residual drop of changing content)
MXHD uint32_t luma_bits_est(const int16_t* co, bool split, int tu4) {
    if (!split) return tu_bits_est(co, 256);
    uint32_t b = 0;
    for (int k = 0; k < 4; ++k) {
        if ((tu4 >> k) & 1)
            for (int j = 0; j < 4; ++j) b += tu_bits_est(co + 64 * k + 16 * j, 16);
        else
            b += tu_bits_est(co + 64 * k, 64);
    }
    return b;
}

// Spatial neighbour motion of a PU (every CU of a P slice is inter, so "available" means inside
// the picture, inside the slice and earlier in decoding order).
struct MvCand {
    bool avail;
    int x, y;
};
// The five spatial neighbours (8.5.3.2.2 / 8.5.3.2.7) of a PU.
struct PuNb {
    MvCand a1, b1, b0, a0, b2;
};

// Merge candidate list (8.5.3.2.2-8.5.3.2.4, MaxNumMergeCand kMaxMergeCand, no TMVP, one
// reference picture): A1, B1 (unless equal to A1), B0 (unless equal to B1), A0 (unless equal to
// A1), B2 (unless equal to A1 or B1, and only while fewer than four), then zero candidates.
MXHD bool mv_eq(MvCand a, MvCand b) { return a.x == b.x && a.y == b.y; }
// Index of vector (mx, my) in the merge list (the first matching entry), -1 if absent.  Walks the
// list without materialising it (no dynamically indexed array: registers only on the GPU).
MXHD int merge_index_of(const PuNb& nb, int mx, int my) {
    int n = 0, found = -1;
    auto add = [&](MvCand c) {
        if (found < 0 && c.x == mx && c.y == my) found = n;
        ++n;
    };
    if (nb.a1.avail) add(nb.a1);
    if (nb.b1.avail && !(nb.a1.avail && mv_eq(nb.b1, nb.a1))) add(nb.b1);
    if (nb.b0.avail && !(nb.b1.avail && mv_eq(nb.b0, nb.b1))) add(nb.b0);
    if (nb.a0.avail && !(nb.a1.avail && mv_eq(nb.a0, nb.a1))) add(nb.a0);
    if (nb.b2.avail && n < 4 && !(nb.a1.avail && mv_eq(nb.b2, nb.a1)) && !(nb.b1.avail && mv_eq(nb.b2, nb.b1)))
        add(nb.b2);
    while (n < kMaxMergeCand) add(MvCand{true, 0, 0});
    return found;
}

// AMVP list (8.5.3.2.6/7, one reference picture so no scaling): A = A0, else A1; B = the first of
// B0, B1, B2; without A the B vector moves into A; duplicates removed; zero padding.
MXHD void amvp_list(const PuNb& nb, int* lx, int* ly) {
    const MvCand a = nb.a0.avail ? nb.a0 : nb.a1;
    const MvCand b = nb.b0.avail ? nb.b0 : (nb.b1.avail ? nb.b1 : nb.b2);
    lx[1] = ly[1] = 0;
    if (a.avail) {
        lx[0] = a.x;
        ly[0] = a.y;
        if (b.avail && (b.x != a.x || b.y != a.y)) {
            lx[1] = b.x;
            ly[1] = b.y;
        }
    } else if (b.avail) {
        lx[0] = b.x;
        ly[0] = b.y;
    } else {
        lx[0] = ly[0] = 0;
    }
}

MXHD int mvd_cost_bits(int d) {
    const int a = d < 0 ? -d : d;
    if (a == 0) return 1;
    if (a == 1) return 3;
    int k = 1, v = a - 2, bits = 3;
    while (v >= (1 << k)) {
        v -= 1 << k;
        ++k;
        ++bits;
    }
    return bits + 1 + k;
}

// Fill type / mvp / mvd of an inter CU (c.mvx/mvy/cbf set) from its neighbours' motion.
// Merge / skip when the CU's vector is in the merge list (mvp_idx then holds merge_idx: the
// first matching entry, the cheapest to signal), else AMVP with the cheaper predictor.
MXHD void decide_inter(CuInfo& c, const PuNb& nb) {
    c.mvp_idx = 0;
    c.mvdx = c.mvdy = 0;
    const int k = merge_index_of(nb, c.mvx, c.mvy);
    if (k >= 0) {
        c.type = c.cbf ? kCuMerge : kCuSkip;
        c.mvp_idx = (uint8_t)k;
        return;
    }
    c.type = kCuAmvp;
    int lx[2], ly[2];
    amvp_list(nb, lx, ly);
    const int c0 = mvd_cost_bits(c.mvx - lx[0]) + mvd_cost_bits(c.mvy - ly[0]);
    const int c1 = mvd_cost_bits(c.mvx - lx[1]) + mvd_cost_bits(c.mvy - ly[1]);
    const int idx = c1 < c0 ? 1 : 0;
    c.mvp_idx = (uint8_t)idx;
    c.mvdx = (int16_t)(c.mvx - lx[idx]);
    c.mvdy = (int16_t)(c.mvy - ly[idx]);
}

// Neighbours of the PU of n x n units (1: a CU16, 2: a CU32) at unit (x, y) of a picture of
// mb_w x mb_h units whose slice starts at CTB first_ctb: A1 (x - 1, y + n - 1), B1 (x + n - 1,
// y - 1), B0 (x + n, y - 1), A0 (x - 1, y + n), B2 (x - 1, y - 1), each available when inside the
// picture, in the slice and earlier in decoding order (z order inside a CTB: e.g. the A0 of a CTB's
// first unit lies in the left CTB and is available, the B0 of its last unit is not).  mv: per unit
// quarter-pel motion, (x, y) at mv[u * stride], mv[u * stride + 1].
MXHD PuNb pu_neighbours(const int16_t* mv, int stride, int x, int y, int n, int mb_w, int mb_h, int first_ctb) {
    const int cw = ctb_cols(mb_w), cur = cpos_of(x, y, cw);
    auto at = [&](int xn, int yn) {
        MvCand c{false, 0, 0};
        if (xn < 0 || yn < 0 || xn >= mb_w || yn >= mb_h) return c;
        if (ctb_of(xn, yn, cw) < first_ctb || cpos_of(xn, yn, cw) >= cur) return c;
        c.avail = true;
        c.x = mv[(size_t)(yn * mb_w + xn) * stride];
        c.y = mv[(size_t)(yn * mb_w + xn) * stride + 1];
        return c;
    };
    PuNb r;
    r.a1 = at(x - 1, y + n - 1);
    r.b1 = at(x + n - 1, y - 1);
    r.b0 = at(x + n, y - 1);
    r.a0 = at(x - 1, y + n);
    r.b2 = at(x - 1, y - 1);
    return r;
}

// Skip / merge / AMVP of the units of CTB (x0, y0) (u[z]: z-order copies, in[z]: inside the
// picture) against the slice's neighbours, then the coding tree: the four units become one CU32
// when all lie inside the picture with one vector and one QP, and the CU32's merge list holds the
// vector (one skip / merge_idx instead of four) or its first unit needs AMVP anyway (one mvd).
// Shared by both encoders (k_hevc_decide: one thread per CTB).
MXHD void decide_ctb(CuInfo* u, const bool* in, const int16_t* mv, int stride, int x0, int y0, int mb_w, int mb_h,
                     int first_ctb) {
    for (int z = 0; z < 4; ++z) {
        if (!in[z]) continue;
        decide_inter(u[z], pu_neighbours(mv, stride, x0 + (z & 1), y0 + (z >> 1), 1, mb_w, mb_h, first_ctb));
        u[z].ct = 1;
    }
    if (!(in[0] && in[1] && in[2] && in[3])) return;
    uint32_t any = 0;
    for (int z = 0; z < 4; ++z) {
        if (u[z].mvx != u[0].mvx || u[z].mvy != u[0].mvy || u[z].qp != u[0].qp) return;
        any |= u[z].cbf;
    }
    const PuNb nb = pu_neighbours(mv, stride, x0, y0, 2, mb_w, mb_h, first_ctb);
    const int k = merge_index_of(nb, u[0].mvx, u[0].mvy);
    if (k < 0 && u[0].type != kCuAmvp) return;
    CuInfo h = u[0];
    h.cbf = (uint8_t)any;
    decide_inter(h, nb);
    for (int z = 0; z < 4; ++z) {
        u[z].type = h.type;
        u[z].mvp_idx = h.mvp_idx;
        u[z].mvdx = h.mvdx;
        u[z].mvdy = h.mvdy;
        u[z].ct = 0;
    }
}

// ---------------------------------------------------------------- deblocking (8.7.2)
// With CTB = CU = PU = TU = 16x16 the only transform / prediction edges on the 8x8 grid are
// the CU edges, and every 4-sample segment of a CU edge shares one boundary strength.
constexpr uint8_t kDbBeta[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  6,  7,
                                 8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 28, 30, 32,
                                 34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64};
constexpr uint8_t kDbTc[54] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1,  1,  1,  1,  1,  1,  1,  1, 1,
                               2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24};

// Luma cbf of the TU of CU c that holds its 4x4 block (bx, by), 0..3 each.
MXHD bool tu_cbf_at(const CuInfo& c, int bx, int by) {
    if (c.tu_split == 2) {
        const int k = (by >> 1) * 2 + (bx >> 1);
        if ((c.tu4 >> k) & 1) return (c.cbf_y16 >> (4 * k + (by & 1) * 2 + (bx & 1))) & 1;
        return (c.cbf_y4 >> k) & 1;
    }
    return c.cbf & 1;
}

// bS of an edge segment between 4x4 block (pbx, pby) of CU p and (qbx, qby) of CU q
// (8.7.2.4): 2 intra, 1 coded luma residual in the TU on either side or a motion difference
// of >= 1 integer sample (one reference picture), else 0.
MXHD int db_bs(const CuInfo& p, int pbx, int pby, const CuInfo& q, int qbx, int qby) {
    if (p.type == kCuIntra || q.type == kCuIntra) return 2;
    if (tu_cbf_at(p, pbx, pby) || tu_cbf_at(q, qbx, qby)) return 1;
    const int dx = p.mvx - q.mvx, dy = p.mvy - q.mvy;
    return (dx >= 4 || dx <= -4 || dy >= 4 || dy <= -4) ? 1 : 0;
}

// One 4-line luma edge segment.  q0 points at the first q sample of line 0, `step` crosses
// the edge (p_i = q0[-(i+1)*step], q_i = q0[i*step]) and `line` advances along it.
MXHD void db_luma_seg(uint8_t* q0, int step, int line, int bs, int qp_p, int qp_q) {
    if (bs == 0) return;
    const int qpl = (qp_p + qp_q + 1) >> 1;
    const int beta = kDbBeta[qpl < 0 ? 0 : (qpl > 51 ? 51 : qpl)];
    int qt = qpl + 2 * (bs - 1);
    qt = qt < 0 ? 0 : (qt > 53 ? 53 : qt);
    const int tc = kDbTc[qt];
    auto P = [&](int k, int i) { return (int)q0[k * line - (i + 1) * step]; };
    auto Q = [&](int k, int i) { return (int)q0[k * line + i * step]; };
    const int dp0 = abs(P(0, 2) - 2 * P(0, 1) + P(0, 0)), dp3 = abs(P(3, 2) - 2 * P(3, 1) + P(3, 0));
    const int dq0 = abs(Q(0, 2) - 2 * Q(0, 1) + Q(0, 0)), dq3 = abs(Q(3, 2) - 2 * Q(3, 1) + Q(3, 0));
    const int dpq0 = dp0 + dq0, dpq3 = dp3 + dq3, dp = dp0 + dp3, dq = dq0 + dq3;
    if (dpq0 + dpq3 >= beta) return;
    auto strong = [&](int k, int dpq) {
        return 2 * dpq < (beta >> 2) && abs(P(k, 3) - P(k, 0)) + abs(Q(k, 0) - Q(k, 3)) < (beta >> 3) &&
               abs(P(k, 0) - Q(k, 0)) < ((5 * tc + 1) >> 1);
    };
    const bool de2 = strong(0, dpq0) && strong(3, dpq3);
    const bool dep = dp < ((beta + (beta >> 1)) >> 3), deq = dq < ((beta + (beta >> 1)) >> 3);
    for (int k = 0; k < 4; ++k) {
        uint8_t* s = q0 + k * line;
        const int p0 = P(k, 0), p1 = P(k, 1), p2 = P(k, 2), p3 = P(k, 3);
        const int q0v = Q(k, 0), q1 = Q(k, 1), q2 = Q(k, 2), q3 = Q(k, 3);
        auto cl = [](int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); };
        if (de2) {
            s[-1 * step] = (uint8_t)cl((p2 + 2 * p1 + 2 * p0 + 2 * q0v + q1 + 4) >> 3, p0 - 2 * tc, p0 + 2 * tc);
            s[-2 * step] = (uint8_t)cl((p2 + p1 + p0 + q0v + 2) >> 2, p1 - 2 * tc, p1 + 2 * tc);
            s[-3 * step] = (uint8_t)cl((2 * p3 + 3 * p2 + p1 + p0 + q0v + 4) >> 3, p2 - 2 * tc, p2 + 2 * tc);
            s[0] = (uint8_t)cl((p1 + 2 * p0 + 2 * q0v + 2 * q1 + q2 + 4) >> 3, q0v - 2 * tc, q0v + 2 * tc);
            s[step] = (uint8_t)cl((p0 + q0v + q1 + q2 + 2) >> 2, q1 - 2 * tc, q1 + 2 * tc);
            s[2 * step] = (uint8_t)cl((p0 + q0v + q1 + 3 * q2 + 2 * q3 + 4) >> 3, q2 - 2 * tc, q2 + 2 * tc);
        } else {
            int d = (9 * (q0v - p0) - 3 * (q1 - p1) + 8) >> 4;
            if (abs(d) >= tc * 10) continue;
            d = cl(d, -tc, tc);
            s[-1 * step] = (uint8_t)clip255(p0 + d);
            s[0] = (uint8_t)clip255(q0v - d);
            if (dep) s[-2 * step] = (uint8_t)clip255(p1 + cl((((p2 + p0 + 1) >> 1) - p1 + d) >> 1, -(tc >> 1), tc >> 1));
            if (deq) s[step] = (uint8_t)clip255(q1 + cl((((q2 + q0v + 1) >> 1) - q1 - d) >> 1, -(tc >> 1), tc >> 1));
        }
    }
}

// Chroma edge lines (bS == 2 only, 8.7.2.5.5); cb_qp_offset = pps_cb/cr_qp_offset.
MXHD void db_chroma_lines(uint8_t* q0, int step, int line, int nlines, int qp_p, int qp_q, int c_qp_offset) {
    const int qpc = chroma_qp(((qp_p + qp_q + 1) >> 1), c_qp_offset);
    int qt = qpc + 2;  // 2 * (bS - 1) with bS = 2
    qt = qt > 53 ? 53 : qt;
    const int tc = kDbTc[qt];
    for (int k = 0; k < nlines; ++k) {
        uint8_t* s = q0 + k * line;
        const int p0 = s[-step], p1 = s[-2 * step], q0v = s[0], q1 = s[step];
        int d = ((((q0v - p0) * 4) + p1 - q1 + 4) >> 3);
        d = d < -tc ? -tc : (d > tc ? tc : d);
        s[-step] = (uint8_t)clip255(p0 + d);
        s[0] = (uint8_t)clip255(q0v - d);
    }
}

// QpY chain of the slice of CTBs [first, end) (8.6.1; quantization groups of 16x16 -- a CU16, or a
// whole CU32): qPY_PRED of a group is the average of the QpY of its left and above groups when
// those lie in the same CTB, else qPY_PREV (the QpY of the previous group in decoding order; the
// slice QP at the slice start and, with WPP, at every CTB row start); a CU that sends cu_qp_delta
// (one with a coded level) has QpY = its QP, any other QpY = qPY_PRED.  Writes qp_pred (the
// entropy coder's delta base) and qpy (deblocking) per unit (raster).
MXHD void slice_qp_chain(const CuInfo* cus, int mb_w, int mb_h, int first, int end, int slice_qp, bool wpp,
                         uint8_t* qp_pred, uint8_t* qpy) {
    const int cw = ctb_cols(mb_w);
    int prev = slice_qp;
    for (int c = first; c < end; ++c) {
        if (wpp && c % cw == 0) prev = slice_qp;
        const int x0 = 2 * (c % cw), y0 = 2 * (c / cw);
        if (cus[y0 * mb_w + x0].ct == 0) {  // CU32: one group, all four units inside
            bool coded = false;
            for (int z = 0; z < 4; ++z) coded |= cus[(y0 + (z >> 1)) * mb_w + x0 + (z & 1)].cbf != 0;
            const int q = coded ? (int)cus[y0 * mb_w + x0].qp : prev;
            for (int z = 0; z < 4; ++z) {
                qp_pred[(y0 + (z >> 1)) * mb_w + x0 + (z & 1)] = (uint8_t)prev;
                qpy[(y0 + (z >> 1)) * mb_w + x0 + (z & 1)] = (uint8_t)q;
            }
            prev = q;
            continue;
        }
        for (int z = 0; z < 4; ++z) {
            const int x = x0 + (z & 1), y = y0 + (z >> 1);
            if (x >= mb_w || y >= mb_h) continue;
            const int i = y * mb_w + x;
            const int qa = (z & 1) ? (int)qpy[i - 1] : prev;
            const int qb = (z & 2) ? (int)qpy[i - mb_w] : prev;
            const int pred = (qa + qb + 1) >> 1;
            const CuInfo& c = cus[i];
            const int q = (c.type != kCuSkip && c.cbf) ? (int)c.qp : pred;
            qp_pred[i] = (uint8_t)pred;
            qpy[i] = (uint8_t)q;
            prev = q;
        }
    }
}

// Deblock the vertical (dir 0) or horizontal (dir 1) CU edge between CU i and its left /
// upper neighbour: rows [r0, r0 + 4) of luma and the matching 2 chroma lines (NV12).
MXHD void db_edge_seg(uint8_t* ry, uint8_t* ruv, int pitch, int ctb_w, const CuInfo* cus, const uint8_t* qpy, int i,
                      int dir, int seg, int c_qp_offset) {
    const int x = i % ctb_w, y = i / ctb_w;
    const int j = dir == 0 ? i - 1 : i - ctb_w;
    const int bs = dir == 0 ? db_bs(cus[j], 3, seg, cus[i], 0, seg) : db_bs(cus[j], seg, 3, cus[i], seg, 0);
    if (!bs) return;
    const int qp_p = qpy[j], qp_q = qpy[i];
    if (dir == 0) {
        db_luma_seg(ry + (size_t)(y * 16 + seg * 4) * pitch + x * 16, 1, pitch, bs, qp_p, qp_q);
        if (bs == 2)
            for (int c = 0; c < 2; ++c)
                db_chroma_lines(ruv + (size_t)(y * 8 + seg * 2) * pitch + x * 16 + c, 2, pitch, 2, qp_p, qp_q,
                                c_qp_offset);
    } else {
        db_luma_seg(ry + (size_t)(y * 16) * pitch + x * 16 + seg * 4, pitch, 1, bs, qp_p, qp_q);
        if (bs == 2)
            for (int c = 0; c < 2; ++c)
                db_chroma_lines(ruv + (size_t)(y * 8) * pitch + x * 16 + seg * 4 + c, pitch, 2, 2, qp_p, qp_q,
                                c_qp_offset);
    }
}

// The internal 8x8 TU edge (vertical dir 0 at x = 8, horizontal dir 1 at y = 8) of a CU
// whose transform tree is split: one PU, so bS is 1 exactly when a TU beside the segment has
// coded luma; luma only (chroma edges lie on the 16-sample grid).
MXHD void db_internal_seg(uint8_t* ry, int pitch, int ctb_w, const CuInfo* cus, const uint8_t* qpy, int i, int dir,
                          int seg) {
    const CuInfo& c = cus[i];
    if (c.tu_split != 2) return;
    // an intra unit's TU edges: Bs 2 (luma only: chroma edges lie on the 16-sample luma grid)
    const bool intra = c.type == kCuIntra;
    const bool coded = intra || (dir == 0 ? (tu_cbf_at(c, 1, seg) || tu_cbf_at(c, 2, seg))
                                          : (tu_cbf_at(c, seg, 1) || tu_cbf_at(c, seg, 2)));
    if (!coded) return;
    const int x = i % ctb_w, y = i / ctb_w, bs = intra ? 2 : 1;
    if (dir == 0)
        db_luma_seg(ry + (size_t)(y * 16 + seg * 4) * pitch + x * 16 + 8, 1, pitch, bs, qpy[i], qpy[i]);
    else
        db_luma_seg(ry + (size_t)(y * 16 + 8) * pitch + x * 16 + seg * 4, pitch, 1, bs, qpy[i], qpy[i]);
}


// ---------------------------------------------------------------- inter transform-tree decision
// ---------------------------------------------------------------- adaptive slice layout (P)
// Entropy-coding cost estimate of a CU in CABAC work units: significance bins up to the
// last position of every coded TU plus a few bins per coded sub-block, on top of the CU
// header.  Used only to balance slices; identical on the CPU and the GPU.
// Serial arithmetic-coder work of a CU in bin tokens (k_hevc_arith runs ~165 ns per token and
// nothing measurable per CTU: tools/hevc_cabac_timing.py).  Least-squares fit over the 16x16 units
// of round-5 4K desktop P pictures (CTB 32 quadtree, 18 Mbps; tools/hevc_session_timing.py --dump,
// tools/hevc_cost_fit.py, profiles/r05_hevc_slices/NOTES.md): a unit without residual 1 token
// (mostly skips: 1.4 measured; merge 5.4, AMVP 12 -- but skip / merge / AMVP are decided after
// the slices are laid out, so the model cannot use them), a coded unit 0.25 per (last + 1) + 13
// per coded sub-block + 3.9 per estimated payload byte - 4.  Replaces round 4's fit (CTB 16),
// which priced a unit without residual at 4 tokens: slices over static areas then held a third
// of their estimate and the slowest slice ran 1.4x the median.
MXHD uint32_t cu_cost(const CuInfo& c) {
    if (!c.cbf) return 1u;
    uint32_t lsum = 0, sb = 0;
    if (c.cbf & 1) lsum += c.last[0] + 1u, sb += (uint32_t)__builtin_popcount(c.csbf_y);
    if (c.cbf & 2) lsum += c.last[1] + 1u, sb += (uint32_t)__builtin_popcount(c.csbf_c[0]);
    if (c.cbf & 4) lsum += c.last[2] + 1u, sb += (uint32_t)__builtin_popcount(c.csbf_c[1]);
    const uint32_t v = (2u * lsum + 104u * sb + 31u * (uint32_t)c.est_bytes) >> 3;
    return v > 5u ? v - 4u : 1u;
}
MXHD uint8_t est_bytes_of(uint32_t bits) {
    const uint32_t b = (bits + 7) >> 3;
    return (uint8_t)(b > 255u ? 255u : b);
}
// est_bytes of a summarised CU from the bits estimate of its final levels (cu_bits_est)
MXHD void set_est_bytes(CuInfo& c, uint32_t bits) { c.est_bytes = c.cbf ? est_bytes_of(bits) : (uint8_t)0; }
// Below this much work per slice, fewer slices: 1536 tokens keep a slice near 0.25 ms; the level's
// slice limit usually binds first at 4K.
constexpr uint32_t kCostPerSlice = 1536;  // EncoderConfig::hevc_slice_cost default
// Largest cu_cost (last+1 <= 256 + 64 + 64, 16 + 4 + 4 sub-blocks, est_bytes <= 255).
constexpr uint32_t kMaxCuCost = ((2u * 384u + 104u * 24u + 31u * 255u) >> 3) - 4u;
// Slices are laid out in whole CTBs: the largest CTB cost (four units)
constexpr uint32_t kMaxCtbCost = 4u * kMaxCuCost;
// Number of slice thresholds for a P picture of total cost T, bounded by the level's slice limit.
// A CTB costlier than the spacing T / S spans several thresholds, so the picture may get fewer
// slices than S: slices start where plan_slice_of changes and are ranked by those starts
// (plan_p_slices; k_hevc_layout compacts the ranks).
// I pictures: each slice is one segment of a CTB row (two per row when the level's slice count
// allows), so the intra wavefront of a slice runs over half the row.  The 16x16-unit column range
// [xb, xe) of the segment holding unit column x, segments seg_w units wide.
MXHD void i_seg_range(int x, int seg_w, int mb_w, int& xb, int& xe) {
    xb = (x / seg_w) * seg_w;
    xe = xb + seg_w < mb_w ? xb + seg_w : mb_w;
}
MXHD int plan_num_slices(uint64_t total, int max_slices, uint32_t cost_per_slice = kCostPerSlice) {
    const uint32_t cps = cost_per_slice > 0 ? cost_per_slice : 1u;
    const uint64_t s = total / cps;
    return s < 1 ? 1 : (s > (uint64_t)max_slices ? max_slices : (int)s);
}
// Slice of a CU whose exclusive cost prefix is `pre`: floor(pre * S / T) -- non-decreasing in
// raster order, so every slice is a raster run and equal-cost runs share the work evenly.
// floor(num / den) for num < 2^52 through one double division and an exact integer fix-up (a
// 64-bit integer division is a ~150-instruction loop on the GPU)
MXHD uint64_t floor_div52(uint64_t num, uint64_t den) {
    uint64_t q = (uint64_t)((double)num / (double)den);
    if (q * den > num) --q;
    else if ((q + 1) * den <= num) ++q;
    return q;
}
MXHD int plan_slice_of(uint64_t pre, uint64_t total, int S) {
    const uint64_t id = floor_div52(pre * (uint64_t)S, total);
    return id >= (uint64_t)S ? S - 1 : (int)id;
}

}  // namespace hevc
}  // namespace mx
